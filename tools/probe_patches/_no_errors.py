# helper for timing probes whose counts are wrong on purpose: the job's
# error words are not raised (the probe's table may lack keys apply meets)
def apply(csrc):
    p = csrc + "/bqsr_capi.cpp"
    s = open(p).read()
    old = "bqsr_status from_err_key(unsigned long long k, int64_t read_base) {"
    assert old in s
    s = s.replace(old, old + "\n  k = kNoError;  // (timing probe: errors not raised)", 1)
    open(p, "w").write(s)
