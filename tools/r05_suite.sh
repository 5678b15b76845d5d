# GPU suite + smoke, then the stationary posterior precision check
bash tools/r05_gputests.sh || exit $?
bash tools/r05_post32chk.sh
