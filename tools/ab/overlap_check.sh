# side-stream overlap at every size >= 2^17: GPU tests, then mesh / power / Bookinfo / 1e9 bench lines
export TMPDIR=/tmp
O=gpurun_out/ovc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
show() { python3 -c "
import json,sys;s=open('$1').read();i=s.index('{\"metric');d,_=json.JSONDecoder().raw_decode(s[i:]);r=d['roofline']
print('$1', d['ms_per_step'], r['kernel'], r['frac'], r['kernel_ms_per_step'])"; }
for c in mesh mesh power; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 --no-h2d > $O/$c.json 2> $O/$c.err || exit 1
  show $O/$c.json
done
timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 --cpu-seconds 0 --no-h2d > $O/book.json 2> $O/book.err || exit 1
show $O/book.json
timeout -k 10 300 python -u bench.py --spans 1e9 --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > $O/mesh1B.json 2> $O/mesh1B.err || exit 1
show $O/mesh1B.json
echo OVC_DONE
