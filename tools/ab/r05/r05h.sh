set -u
mkdir -p gpurun_out/r05h
bash tools/ab_run.sh r05h_d "--config c5 --rng seeded --stream-ring doubles" cur \
 && bash tools/ab_run.sh r05h_b "--config c5 --rng seeded" cur mj8 mj16 \
 && bash tools/ab_run.sh r05h_d2 "--config c5 --rng seeded --stream-ring doubles" cur \
 && bash tools/ab_run.sh r05h_b2 "--config c5 --rng seeded" cur mj8 mj16 \
 && bash tools/ab_run.sh r05h_s "--config c5 --rng stream" r4launch nofold scan3 cur r4launch nofold scan3 cur \
 && bash tools/ab_run.sh r05h_p "--config c5" cur cur
