# occupancy probe (counts stay correct): only the first W of a workgroup's 16
# waves walk reads (W from the env var PROBE_WAVES at build time: the patch
# hard-codes it), the others only join the barriers -- if the kernel time
# scales with 16 / W the walk is latency-bound per wave, if it stays flat a
# per-CU resource (TA / L1 / LDS) is the bound
import os, sys
W = int(os.environ.get("PROBE_WAVES", "8"))
p = sys.argv[1] + "/bqsr_observe_lean.hip"
s = open(p).read()
old = "  for (int64_t g0 = p0 + 64 * wave; g0 < p1; g0 += 64 * kWaves) {"
assert old in s
s = s.replace(old, "  for (int64_t g0 = p0 + 64 * wave; wave < %d && g0 < p1; g0 += 64 * %d) {" % (W, W), 1)
open(p, "w").write(s)
