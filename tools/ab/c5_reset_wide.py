# C5: k_env_reset_list_wide with the 128x128 shape at compile time (shifts and masks
# for the cell index and torus wraps): apply c5_reset_wide.patch, then build "rw" from
# the tree (rw_base = the build without it).  Measured +0.6-0.9% on C5 (64.8-65.0 vs
# 64.4 M, same box), parity green; not kept (below the bench's run-to-run spread).
VARIANTS = {"rw": []}
