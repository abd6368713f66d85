# summarise a gpu_full.sh run: test tail and one line per bench
tag=$1
tail -2 gpurun_out/$tag/pytest.log
for f in gpurun_out/$tag/bench*.log; do
  python -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('%-28s %8.1f Mrays/s %8.1f ms/step frac %.4f  %s' % ('$f'.split('/')[-1], d['value'], d['ms_per_step'], r['frac'], r['launch'][:60]))"
done
