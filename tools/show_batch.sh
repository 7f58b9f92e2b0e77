#!/bin/bash
# Print the results of tools/gpu_batch.sh merged back under gpurun_out/.
cat gpurun_out/decode_ablate.log 2>/dev/null
tail -2 gpurun_out/pytest_gpu.log 2>/dev/null
tail -2 gpurun_out/stamps16.log 2>/dev/null
for C in 1 16; do
  [ -f gpurun_out/b_c${C}_f0.log ] && python -c "
import json; d=json.loads(open('gpurun_out/b_c${C}_f0.log').read().strip().splitlines()[-1])
print($C, d['value'], d['ms_per_step'], d['step_roofline']['frac'], d['roofline']['kernel'], d['roofline']['frac'], d['stages_ms'])"
done
cat gpurun_out/bench_aggregate.log 2>/dev/null
[ -n "$1" ] && cat gpurun_out/prof_$1/summary.json gpurun_out/prof_$1/host_rate.jsonl 2>/dev/null
true
