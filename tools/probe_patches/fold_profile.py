# profile build of the expectedMismatch fold (device printf of cycles per
# segment / chain phase, as profiles/r04y_cfg2_fold_profile.txt): the
# instrumentation kept as a patch (fold_profile.diff), built with -DBQSR_FOLD_PROFILE
import os, subprocess, sys
csrc = sys.argv[1]
d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fold_profile.diff")
subprocess.run(["patch", "-s", "-p3", "-d", csrc, "-i", d], check=True)
p = csrc + "/bqsr_fold.hip"
s = open(p).read()
open(p, "w").write("#define BQSR_FOLD_PROFILE 1\n" + s)
