set -o pipefail
mkdir -p gpurun_out/hwq
for rep in 1 2; do
  for q in ${QS:-4 8 16}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline-only --steps 60 > gpurun_out/hwq/q$q.$rep.json 2> gpurun_out/hwq/q$q.$rep.err || { tail -5 gpurun_out/hwq/q$q.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/hwq/q$q.$rep.json "q=$q"
  done
done
