set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for t in _old .; do
    (cd $t && timeout -k 10 300 python bench.py --mode fwd --steps 10 --warmup 3 --no-cpu-baseline --no-roofline-step > /tmp/fwd.json 2>/tmp/fwd.err) || { echo "fwd $t failed"; tail -5 /tmp/fwd.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('/tmp/fwd.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$t #$i"
  done
done
