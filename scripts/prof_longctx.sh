#!/bin/bash
# Decode-step timeline at long contexts (TTSD shape, n_vq 16): rocprofv3 kernel trace of a
# short bench run per prompt length.  Writes gpurun_out/longctx/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/longctx
mkdir -p $O
export TMPDIR=/tmp
for tt in ${TEXT_TOKENS:-2000 8000}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/plc$tt -o run --output-format csv -- \
      python3 bench.py --config ttsd --text-tokens $tt --decode-steps ${DSTEPS:-64} --steps 1 --warmup 0 \
      --no-cpu-baseline --no-roofline --no-codec > $O/bench_$tt.json 2> $O/err_$tt.txt
  rc=$?; echo "text_tokens=$tt rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/err_$tt.txt; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/bench_$tt.json'));print('ms/step', d['ms_per_decode_step'], 'prefill', d.get('prefill_ms'))"
  f=$(find /tmp/plc$tt -name "*kernel_trace.csv" | head -1)
  KTRACE_SEQ=${SEQ:-14} python3 scripts/ktrace.py $f > $O/timeline_$tt.txt
  head -24 $O/timeline_$tt.txt
done
