# fp16x3 update from dataflow-written planes vs the in-register split (tools/upd32_bench.cpp):
# checksums must match, timing per launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05pl; mkdir -p $O
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -x hip"
$H tools/upd32_bench.cpp -o /tmp/upd_pl || exit 1
for K in 0 3 5; do
  timeout -k 5 120 /tmp/upd_pl 64 $K 10 det || exit $?
  UPD_PLANES=1 timeout -k 5 120 /tmp/upd_pl 64 $K 10 det || exit $?
done 2>&1 | tee $O/pl.txt
timeout -k 10 300 python -u tools/ab_knob.py APM_PLANES 0 1 --reps 3 2>&1 | tee $O/ab_planes.txt
