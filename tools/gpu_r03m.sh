# Round 3 profiles: bench line + kernel-trace stats + HBM counter passes, then the other BASELINE configurations.
set -e
bash tools/profile_round.sh r03
bash tools/gpu_configs.sh
