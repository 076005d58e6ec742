COMMIT=$1 bash tools/final_round.sh r04 || exit 1
