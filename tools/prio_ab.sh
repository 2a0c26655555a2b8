# A/B of the pipelined step's stream priorities (CAPMI_PIPE_PRIO: default encoder high / decoder low since round 6; dec, equal)
set -e
: > gpurun_out/prio_ab.txt
for p in default dec equal default dec equal; do
  CAPMI_PIPE_PRIO=$p timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/prio.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/prio.log') if l.startswith('{')][-1]); print('$p', d['value'], d['ms_per_step'])" >> gpurun_out/prio_ab.txt
done
