# A/B of the hybrid data-parallel + stream-K schedule (CAPMI_SK_HYBRID=0|1): GEMM tests, per-shape
# timings (plan printed), then the headline bench with each
set -e
out=gpurun_out/hybrid_ab.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hybrid_test.log 2>&1
for s in l3c3 l2c3 l1c3 ds1 l1c1 l1c2 l2c1 ds2 l3c2 l4c3; do
  for h in 0 1; do echo "h$h $(CAPMI_SK_HYBRID=$h timeout -k 10 60 python tools/gemm_one.py --shape $s --reps 100 2>&1 | grep -E 'plan|TFLOP' | tr '\n' ' ')" >> $out; done
done
for h in 0 1 0 1; do
  CAPMI_SK_HYBRID=$h timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/hybrid_bench.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/hybrid_bench.log') if l.startswith('{')][-1]); r=d['roofline']; print('bench h$h', d['value'], d['ms_per_step'], r['kernel'], r['achieved'], r['conv_family']['conv_ms_per_step'])" >> $out
done
