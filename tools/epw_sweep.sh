set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/envtests.txt 2>&1
for e in 1 4 8; do
  for n in 4096 32768; do
    MSENV_EPW=$e timeout -k 10 120 python bench.py --no-cpu-baseline --ppo-updates 0 --envs $n > gpurun_out/b_$e_$n.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/b_$e_$n.json'));print('epw $e n $n value %.3g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac']))"
  done
done
MSENV_EPW=4 timeout -k 10 200 python tools/diag_step.py > gpurun_out/diag4096_e4.txt 2>&1
