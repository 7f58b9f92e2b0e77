set -e
O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2; do
timeout -k 10 100 python bench.py --no-cpu-baseline > $O/new$r.json 2>&1
timeout -k 10 100 python bench.py --no-cpu-baseline --fork > $O/newfork$r.json 2>&1
timeout -k 10 100 python tools/ab/bench_old.py --no-cpu-baseline > $O/old$r.json 2>&1
done
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['stages_ms'])"; done
