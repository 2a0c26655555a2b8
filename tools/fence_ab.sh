# A/B of scheduling fences in the fp32 conv k-step (CAPMI_KSTEP_FENCE / CAPMI_LOAD_FENCE builds in ablibs/)
# (the CAPMI_KSTEP_FENCE / CAPMI_LOAD_FENCE macros were folded into the kernel after this measurement)
set -e
out=gpurun_out/fence_ab.txt; : > $out
for v in ablibs/*.so; do
  for s in l3c2 l3c1 l3c3 l4c2 l2c2 l1c2; do
    echo "$v $(CAPMI_LIB=$PWD/$v timeout -k 10 60 python tools/gemm_one.py --shape $s --reps 100 2>&1 | grep TFLOP)" >> $out
  done
done
for v in ablibs/*.so ablibs/*.so; do
  CAPMI_LIB=$PWD/$v timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/fence_bench.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/fence_bench.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v bench', d['value'], d['ms_per_step'], r['achieved'], r['conv_family']['conv_ms_per_step'])" >> $out
done
