# A/B of the narrow (16-channel) BN finalize for 65..256 slices (CAPMI_BNF_NARROW=0|1)
set -e
out=gpurun_out/bnf_ab.txt; : > $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread -k "bn_finalize or encoder" > gpurun_out/bnf_test.log 2>&1
for h in 0 1; do echo "narrow$h $(CAPMI_BNF_NARROW=$h timeout -k 10 60 python tools/bnf_time.py 2>&1 | grep bn_finalize | tr '\n' ' ')" >> $out; done
for h in 0 1 0 1; do
  CAPMI_BNF_NARROW=$h timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/bnf_bench.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bnf_bench.log') if l.startswith('{')][-1]); print('bench narrow$h', d['value'], d['ms_per_step'])" >> $out
  CAPMI_BNF_NARROW=$h timeout -k 10 150 python bench.py --sequential --steps 30 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/bnf_bench.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bnf_bench.log') if l.startswith('{')][-1]); print('seq narrow$h', d['value'], d['ms_per_step'])" >> $out
done
