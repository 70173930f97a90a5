# quick GPU check of the env path: parity tests + env-step bench lines + k_step phase stamps
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py tests/test_rl_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/envtests.txt 2>&1
for n in 4096 32768; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --ppo-updates 0 --envs $n > gpurun_out/b_$n.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/b_$n.json'));print('n $n value %.4g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac']))"
done
for b in 9x9x10 30x16x99; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --ppo-updates 0 --envs 8192 --board $b > gpurun_out/b_$b.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/b_$b.json'));print('$b n 8192 value %.4g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac']))"
done
timeout -k 10 200 python tools/diag_step.py --board 9x9x10 --envs 8192 > gpurun_out/diag9.txt 2>&1
python -c "import json;d=json.load(open('gpurun_out/b_4096.json'))['multistep'];print('multistep 4096 value %.4g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_per_step'],d['roofline']['frac']))"
python -c "import json;d=json.load(open('gpurun_out/b_32768.json'))['multistep'];print('multistep 32768 value %.4g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_per_step'],d['roofline']['frac']))"
python -c "import json;d=json.load(open('gpurun_out/b_9x9x10.json'))['multistep'];print('multistep 9x9 value %.4g ms/step %.4f kern_ms %.4f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_per_step'],d['roofline']['frac']))"
