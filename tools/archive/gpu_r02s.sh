# round 2: packet slots in flight against phase size (C2: 1e7 packets per step; C5: dust phases of 4e5
# packets per wavelength with 1/10 and 1/3 stages); default 2^23
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/slots_sweep.txt; : > $out
for cfg in c2 c5; do
  for s in 0 262144 524288 1048576 2097152 4194304; do
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --slots $s > gpurun_out/sw.log 2>&1 || { echo "fail $cfg $s"; exit 1; }
    python -c "
import json
for l in open('gpurun_out/sw.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; c=d['config']
        print('$cfg slots=$s', '%.4g pkt/s'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'iters', c['iterations'], 'trace %.3f x %d'%(r['launch_ms_avg'], r['launches_per_step']))" >> $out
    tail -1 $out
  done
done
