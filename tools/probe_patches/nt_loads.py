# A/B variant (counts unchanged): the per-base passes' bulk loads -- quals,
# base codes, slot-bitmap words of bqsr_observe_lean, quals and codes of the
# apply walk -- as nontemporal (global_load ... nt: streamed once, no
# allocation in the near caches)
import sys
d = sys.argv[1]
def patch(f, pairs):
    p = d + "/" + f
    s = open(p).read()
    for old, new in pairs:
        assert old in s, old
        s = s.replace(old, new, 1)
    open(p, "w").write(s)
patch("bqsr_internal.h", [("struct alignas(8) ReadInfo {",
    "typedef unsigned int NtU4 __attribute__((ext_vector_type(4)));\n"
    "typedef unsigned int NtU3 __attribute__((ext_vector_type(3), aligned(4)));\n"
    "__device__ __forceinline__ uint4 nt_u4(const void* p) { const NtU4 v = __builtin_nontemporal_load((const NtU4*)p); return make_uint4(v.x, v.y, v.z, v.w); }\n"
    "__device__ __forceinline__ uint3 nt_u3(const void* p) { const NtU3 v = __builtin_nontemporal_load((const NtU3*)p); return make_uint3(v.x, v.y, v.z); }\n"
    "__device__ __forceinline__ uint64_t nt_u64(const uint64_t* p) { return __builtin_nontemporal_load(p); }\n"
    "struct alignas(8) ReadInfo {")])
patch("bqsr_observe_lean.hip", [
    ("qs[i] = lv ? *(const uint4*)(qp + o0) : make_uint4(0, 0, 0, 0);", "qs[i] = lv ? nt_u4(qp + o0) : make_uint4(0, 0, 0, 0);"),
    ("? *(const uint3*)(P.rd.bases + ((n0 >> 3) << 2)) : make_uint3(0, 0, 0);", "? nt_u3(P.rd.bases + ((n0 >> 3) << 2)) : make_uint3(0, 0, 0);"),
    (": P.sbits[(s0 >> 5) + w];", ": nt_u64(P.sbits + (s0 >> 5) + w);"),
])
patch("bqsr_kernels.hip", [
    ("    v.qs = *(const uint4*)(P.rd.qual + x.slot + o0);\n    if (!(x.fl & kInfoPass)) v.cr = chunk_raw(P.rd, chunk_n0(x, o0));",
     "    v.qs = nt_u4(P.rd.qual + x.slot + o0);\n    if (!(x.fl & kInfoPass)) { const int64_t n0 = chunk_n0(x, o0); v.cr = n0 >= 0 ? nt_u4(P.rd.bases + (n0 >> 1)) : make_uint4(0, 0, 0, 0); }"),
])
