# A/B variant (counts unchanged): each wavefront step of bqsr_observe_lean
# touches one dword per cache line of its NEXT step's quals / codes / bitmap
# span (estimated from lane 0's slot and span: 64 x 16 reads ahead) right
# after issuing this step's loads, so the next step's lines are in L2 /
# MALL when its own loads reach them -- a test of whether the L1's misses to
# HBM (TCP pending stalls 68 % of cycles) bound the walk
import sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = """#pragma clang loop unroll(full)
      for (int i = 0; i < kLeanSub; ++i) {
        const int j = j0 + kChunk * i;"""
assert old in s
new = """      uint32_t pfa = 0, pfb = 0;
      {
        const uint32_t sl = __builtin_amdgcn_readfirstlane((uint32_t)x.slot), sh = __builtin_amdgcn_readfirstlane((uint32_t)(x.slot >> 32));
        const uint32_t sp = __builtin_amdgcn_readfirstlane((uint32_t)slot_span(x.lq, x.ls));
        const uint64_t nx = (((uint64_t)sh << 32) | sl) + (uint64_t)sp * 64u * kWaves;
        if (nx + 8192 < (uint64_t)P.rd.n_slots) {
          pfa = *(const volatile uint32_t*)(P.rd.qual + nx + 128 * lane);
          if (lane < 32) pfb = *(const volatile uint32_t*)(P.rd.bases + nx / 2 + 128 * lane);
          else if (lane < 48) pfb = *(const volatile uint32_t*)((const uint8_t*)(P.sbits + (nx >> 5)) + 128 * (lane - 32));
        }
      }
#pragma clang loop unroll(full)
      for (int i = 0; i < kLeanSub; ++i) {
        const int j = j0 + kChunk * i;"""
s = s.replace(old, new, 1)
old2 = """        }
      }
    }
  }
  __syncthreads();
  // ---- the window -> the piece's slab"""
assert old2 in s
new2 = """        }
      }
      asm volatile("" ::"v"(pfa), "v"(pfb));
    }
  }
  __syncthreads();
  // ---- the window -> the piece's slab"""
s = s.replace(old2, new2, 1)
open(p, "w").write(s)
