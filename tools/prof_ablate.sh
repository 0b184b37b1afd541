bash tools/profile_round.sh r01 && bash tools/ablate.sh
