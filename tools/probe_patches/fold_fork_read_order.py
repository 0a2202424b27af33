# A/B variant (results unchanged): a read-order batch's expectedMismatch fold
# forked after prep onto the batch's second stream as bucketed batches do:
# bqsr_fold_hist makes the fold's per-block qual histograms from prep's
# (deferred) trims beside the lean observe kernel, which then writes none
# (verdict r05 #4: take the fold off cfg2's critical path)
import sys
d = sys.argv[1]
def patch(f, pairs):
    p = d + "/" + f
    s = open(p).read()
    for old, new in pairs:
        assert old in s, old
        s = s.replace(old, new, 1)
    open(p, "w").write(s)
patch("bqsr_observe_lean.hip", [
    ("  if (ident)\n    for (int k = tid; k < kQBins; k += blockDim.x) P.hq_block",
     "  if (ident && P.hq_block)\n    for (int k = tid; k < kQBins; k += blockDim.x) P.hq_block"),
])
patch("bqsr_capi.cpp", [
    ("    if (!lean) {\n      if (!b->side) {", "    if (true) {\n      if (!b->side) {"),
    ("    P.hq_block = b->d_hq;", "    P.hq_block = lean ? nullptr : b->d_hq;"),
    ("    if (b->bucketed) {  // the observe kernel did not walk the fold's blocks in read order: their histograms",
     "    if (true) {  // the observe kernel did not walk the fold's blocks in read order: their histograms"),
])
