# 256x256 quad-tile fp16x3 update vs the 128-row kernel (tools/upd32_bench.cpp): checksums must
# match; timing per launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05q; mkdir -p $O
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -x hip"
$H tools/upd32_bench.cpp -o /tmp/upd_q || exit 1
for K in 0 3 5; do
  UPD_PLANES=1 timeout -k 5 120 /tmp/upd_q 64 $K 10 det || exit $?
  UPD_PLANES=1 UPD_Q256=1 timeout -k 5 120 /tmp/upd_q 64 $K 10 det || exit $?
done 2>&1 | tee $O/q.txt

