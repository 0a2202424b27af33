# A/B variant (results unchanged): the apply walk's qual and base-code loads
# nontemporal (global_load ... nt), the observe kernels untouched -- round 6
# nt_loads.py measured apply -1 % with observe's loads nt as well
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
    "__device__ __forceinline__ uint4 nt_u4(const void* p) { const NtU4 v = __builtin_nontemporal_load((const NtU4*)p); return make_uint4(v.x, v.y, v.z, v.w); }\n"
    "struct alignas(8) ReadInfo {")])
patch("bqsr_kernels.hip", [
    ("    v.qs = *(const uint4*)(P.rd.qual + x.slot + o0);\n    if (!(x.fl & kInfoPass)) v.cr = chunk_raw(P.rd, chunk_n0(x, o0));",
     "    v.qs = nt_u4(P.rd.qual + x.slot + o0);\n    if (!(x.fl & kInfoPass)) { const int64_t n0 = chunk_n0(x, o0); v.cr = n0 >= 0 ? nt_u4(P.rd.bases + (n0 >> 1)) : make_uint4(0, 0, 0, 0); }"),
])
