set -o pipefail
mkdir -p gpurun_out/abb
for r in 1 2 3; do
  for v in bench bench_prev; do
    timeout -k 10 300 python $v.py --no-cpu-baseline --no-variants --steps 20 --warmup 3 > gpurun_out/abb/${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('persons_per_s'), d.get('frames_over_caps'), d['config']['parallelism'][:40])" gpurun_out/abb/${v}_$r.log $v | tee -a gpurun_out/abb/summary.log
  done
done
