set -u
# round-5 final session: tools/final_round.sh r05q a, then r05q b (two gpurun calls)
bash tools/final_round.sh r05q "$1"
