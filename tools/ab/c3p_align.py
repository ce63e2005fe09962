# C3 packed views: does the env's view alignment matter?  Timing-only probe: each env
# writes 1 088 of its 1 089 cells at env stride 1 088 (2 176 B = 17 x 128 B, every
# env's first cell 128-B aligned) instead of 1 089 at 2 178 B (neighbouring envs,
# on different XCDs, share a partly written line and 32-B sector).
F = "sl_bits.hip"
OLD = """    uint16_t *o = lfx.obs_out + b * (int64_t)nv;
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    if (small) {
        for (int i = lane; i < nv; i += 64) {"""
NEW = """    uint16_t *o = lfx.obs_out + b * (int64_t)(nv - 1);
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    if (small) {
        for (int i = lane; i < nv - 1; i += 64) {"""
SHORT = """    uint16_t *o = lfx.obs_out + b * (int64_t)nv;
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    if (small) {
        for (int i = lane; i < nv - 1; i += 64) {"""
VARIANTS = {"al_base": [], "al_aligned": [(F, OLD, NEW)], "al_short": [(F, OLD, SHORT)]}
