cd "$GRAFT_REPO_ROOT"
for e in "MTTS_NONE=1" "MTTS_NW=4,4,4,4,0" "MTTS_NW=16,16,16,16,0" "MTTS_U=8,8,8,8,0" "MTTS_GEMV_RT2=0"; do
  echo "$e $(env $e timeout -k 10 120 python3 scripts/gemv_probe.py 32 2>&1 | tail -1)"
done
echo "B1 $(timeout -k 10 120 python3 scripts/gemv_probe.py 1 2>&1 | tail -1)"
echo "B4 $(timeout -k 10 120 python3 scripts/gemv_probe.py 4 2>&1 | tail -1)"
