# C3: the 64x64 pool planes reordered so the eleven start planes the scores read fill
# six DMA rows (was seven), with the pristine-goal colour rows (two more rows, planes_ok
# bit 5) switched off -- the layout change alone (pk6) against the tree as built.
F = "sl_bits.hip"
VARIANTS = {"pk6": [(F, "    const bool gpool = pok == 6 && (pok_all & 32) && roll >= 0 && fx.pool.goal_planes;",
                        "    const bool gpool = false;")]}
