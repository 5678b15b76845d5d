# determinism of the Newton update microbenchmark across processes (tools/upd32_bench.cpp)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -x hip"
$H tools/upd32_bench.cpp -o /tmp/upd_new || exit 1
for K in 0 3; do for r in 1 2; do timeout -k 5 120 /tmp/upd_new 64 $K 3 || exit $?; done; done | tee $O/det.txt
