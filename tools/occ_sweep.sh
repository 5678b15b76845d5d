set -e
for pad in 0 12288 30720; do
  APM_LOOKAHEAD=0 APM_UPD_LDS_PAD=$pad timeout -k 10 120 python3 tools/time_theta.py --batch 64 --reps 2 > gpurun_out/occ_$pad.log 2>&1
done
