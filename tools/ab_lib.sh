# development: A/B the current libapm.so against an older build on the same box
set -e
echo "== old (lookahead off)"; APM_LOOKAHEAD=0 APM_LIB=tools/_oldlib/libapm_b2d8f9b.so timeout -k 10 120 python3 tools/time_theta.py --batch 64 --reps 2 | grep "rep 1\|update"
echo "== old (lookahead on)"; APM_LIB=tools/_oldlib/libapm_b2d8f9b.so timeout -k 10 120 python3 tools/time_theta.py --batch 64 --reps 2 | grep "rep 1\|update"
echo "== new"; timeout -k 10 120 python3 tools/time_theta.py --batch 64 --reps 2 | grep "rep 1\|update"
echo "== new, no fuse"; APM_FUSE_DIAG=0 timeout -k 10 120 python3 tools/time_theta.py --batch 64 --reps 2 | grep "rep 1\|update"
