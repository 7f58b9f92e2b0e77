set -e
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
for cfg in "1 -1" "2 0" "2 -1"; do
  set -- $cfg; L=$1; PR=$2; D=/tmp/tr${L}_$PR
  timeout -k 10 240 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes $L --c-priority $PR --no-cpu-baseline > $O/tr${L}_$PR.json 2> $O/tr${L}_$PR.err
  python3 tools/timeline.py $D --dump 24 > $O/timeline_${L}_$PR.txt
  du -sh $D
  rm -rf $D
done
timeout -k 10 120 python tools/select_stamps.py 16 > $O/stamps16.log 2>&1
ls -la $O
