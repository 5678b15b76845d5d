# Counter passes of the fp16x3 trailing update alone (tools/upd32_bench.cpp, K = 0, 64 chains):
# the 128-row super-tile kernel on planes (ROLE 2) and the 256x256 quad-tile kernel. One rocprofv3
# run per pass and variant, each under its own time limit; summaries by tools/pmc_kernels.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_upd; mkdir -p $O
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -x hip"
$H tools/upd32_bench.cpp -o /tmp/upd_q || exit 1
export UPD_PLANES=1
run() {  # variant(0/1), name, counters...
  local v=$1; local name=$2; shift 2
  UPD_Q256=$v timeout -s KILL 60 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/q$v/$name -o run -- /tmp/upd_q 64 0 3 > $O/q$v.$name.log 2>&1
  local rc=$?
  echo "variant $v pass $name: exit $rc"
  return $rc
}
for v in 0 1; do
  run $v mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
  run $v insts SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
  run $v waits SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU || exit $?
  run $v fetch FETCH_SIZE || exit $?
  run $v write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $?
  run $v ta TA_BUSY_avr TA_TA_BUSY_sum || run $v ta TA_BUSY_avr || true
  F=""
  for p in mfma insts waits fetch write ta; do
    c=$(find $O/q$v/$p -name '*counter_collection.csv' 2>/dev/null | head -1)
    [ -n "$c" ] && F="$F $c"
  done
  python3 tools/pmc_kernels.py --match k_chol_update32_t128 --match k_chol_update32_q256 $F > $O/summary_q$v.txt 2>&1
done
find $O -name '*.csv' -delete
echo done
