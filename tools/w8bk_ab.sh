# A/B of the k-tile depth of the 512-thread fp32 conv form (CAPMI_W8_BK=32|64): parity tests with
# (CAPMI_W8_BK was removed after this measurement; the knob lives in git history)
# 64, per-shape timings, then the headline bench with each
set -e
mkdir -p gpurun_out; : > gpurun_out/w8bk_ab.txt
CAPMI_W8_BK=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "512_thread or auto_tile" > gpurun_out/w8bk_test.log 2>&1
for s in l1c3 ds1 l2c1 l2c2s l2c2 l3c1 l3c2 ds3 l4c1 l4c2 l4c3 ds4; do
  for b in 32 64; do echo "bk$b $(CAPMI_W8_BK=$b timeout -k 10 60 python tools/gemm_one.py --shape $s --tile 4 2>&1 | grep TFLOP)" >> gpurun_out/w8bk_ab.txt; done
done
for b in 32 64 32 64; do
  CAPMI_W8_BK=$b timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/w8bk_bench.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/w8bk_bench.log') if l.startswith('{')][-1]); r=d['roofline']; print('bench bk$b', d['value'], d['ms_per_step'], r['kernel'], r['achieved'], r['conv_family']['conv_ms_per_step'])" >> gpurun_out/w8bk_ab.txt
done
