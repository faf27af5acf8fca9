# round 2: stage times of the device density sampling (C3 setup)
set -o pipefail
cd $GRAFT_REPO_ROOT
SKIRT_AMD_SETUP_TIMES=1 timeout -k 10 300 python -c "
import skirt_amd as S, time
t=time.time(); S.Simulation('tests/golden/ski/pan_oct.ski', setup_device=0); print('warm-up load (HIP init) %.2f s' % (time.time()-t))
print('device'); S.Simulation('benchmarks/c3_oct128.ski', setup_device=0)
" > gpurun_out/setup_times2.log 2>&1; echo rc=$?
