# timing probe (wrong counts): bqsr_observe_lean's per-step loads of quals,
# base codes and bitmap words made contiguous across the wave's lanes (lane l
# reads 16 B at 16 (l + 64 i) of a block near its read) instead of at its
# own read's slots: what the lane-per-read access pattern costs.  The loaded
# quals are other reads' quals (padding zeros read as Q38: every key the
# table sees exists) and the
# loaded bitmap words are cleared at run time (rows_all is 1 on cfg2).
import sys
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)
rep("        qs[i] = lv ? *(const uint4*)(qp + o0) : make_uint4(0, 0, 0, 0);",
    "        { uint4 t = lv ? *(const uint4*)(P.rd.qual + min(x.slot & ~(uint64_t)16383, (uint64_t)P.rd.n_slots - 16384) + 16 * (lane + 64 * i)) : make_uint4(0, 0, 0, 0);\n"
    "          auto fz = [](uint32_t v) { const uint32_t z = ((v - 0x01010101u) & ~v & 0x80808080u) >> 7; return v + z * 38u; };\n"
    "          qs[i] = make_uint4(fz(t.x), fz(t.y), fz(t.z), fz(t.w)); }")
rep("        cr[i] = (lv && full && n0 >= 0) ? *(const uint3*)(P.rd.bases + ((n0 >> 3) << 2)) : make_uint3(0, 0, 0);",
    "        cr[i] = (lv && full && n0 >= 0) ? *(const uint3*)(P.rd.bases + min(x.slot & ~(uint64_t)16383, (uint64_t)P.rd.n_slots - 16384) / 2 + 12 * (lane + 64 * i)) : make_uint3(0, 0, 0);")
rep(": P.sbits[(s0 >> 5) + w];",
    ": (P.sbits[min(s0 >> 5 & ~(uint64_t)1023, (uint64_t)P.rd.n_slots / 32 - 1024) + lane + 64 * w] & (uint64_t)(P.rows_all - 1));")
open(p, "w").write(s)
sys.path.insert(0, __import__("os").path.dirname(__file__))
import _no_errors
_no_errors.apply(sys.argv[1])
