# The bit-ring generator's waves at issue priority 3 (round 6: with the step stream's
# kernels shorter, the look-ahead's blocks set the pace of a seeded C5 step)
OLD = """k_mt_gen_bits(MtArgs a) {
"""
NEW = """k_mt_gen_bits(MtArgs a) {
    __builtin_amdgcn_s_setprio(3);
"""
VARIANTS = {"mt_prio": [("sl_mt.hip", OLD, NEW)]}
