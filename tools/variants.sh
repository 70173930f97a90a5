cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for a in "--tape 0" "--tape 1" "--tape 0 --envs 32768" "--tape 1 --envs 32768" "--tape 0 --diag-no-obs" "--tape 1 --diag-no-obs" "--board 9x9x10 --envs 8192" "--board 30x16x99 --envs 1024" "--board 30x16x99 --envs 8192"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $a > gpurun_out/v.log 2>&1 || { echo "FAIL $a"; cat gpurun_out/v.log | tail -5; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('$a', '%.1fM/s'%(d['value']/1e6), 'kern %.1fus'%(d['roofline']['kernel_ms']*1e3), 'step %.1fus'%(d['ms_per_step']*1e3), 'frac %.3f'%d['roofline']['frac'])"
done
