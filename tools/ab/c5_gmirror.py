# C5: the goals' six planes (0, 3, 4, 9-11) kept in the mirror and read back from it
# for goals of the usual cell types (spawn_flags bits 1 and 3 clear) -- the tree as
# committed with it; gm_base is the previous build (variants/gm_base.so, copied).
VARIANTS = {"gm": []}
