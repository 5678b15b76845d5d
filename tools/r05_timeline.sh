# kernel trace of two stationary 64-chain theta-calls; phase split and one Newton iteration's
# timeline (tools/theta_phases.py, tools/newton_timeline.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05tl; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/time_theta.py --batch 64 --reps 2 --no-prof --theta-file profiles/r04_stationary_thetas.npy > $O/run.log 2>&1 || exit $?
T=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 tools/theta_phases.py $T > $O/phases.txt 2>&1
python3 tools/newton_timeline.py $T --iter 3 > $O/iter3.txt 2>&1
python3 tools/newton_timeline.py $T --iter 0 --max-rows 0 > $O/iter0.txt 2>&1
gzip -c $T > $O/trace.csv.gz
find $O/tr -name '*.csv' -delete
echo done
