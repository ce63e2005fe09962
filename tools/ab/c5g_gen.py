# C5 seeded: threads per generating workgroup (k_mt_gen<NT>): one wave holds one wave
# slot per block beside the step kernel, at a longer latency per round.
F = "sl_mt.hip"
VARIANTS = {"gen%d" % n: [(F, "constexpr int kGenThreads = 256;", "constexpr int kGenThreads = %d;" % n)]
            for n in (64, 128, 256)}
