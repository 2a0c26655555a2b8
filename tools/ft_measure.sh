tools/gpu_steps.sh \
  "300|fttest|python -u -m pytest tests/test_gpu_finetune.py -x -q -s --timeout 200 --timeout-method thread -k shallow" \
  "300|ftbench|python bench.py --config glove_finetune --steps 10 --warmup 2" \
  "300|ftbench_eager|python bench.py --config glove_finetune --steps 10 --warmup 2 --sequential --eager --no-cpu-baseline"
