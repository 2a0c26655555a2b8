tools/gpu_steps.sh \
 "200|t_x3|python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread" \
 "120|b_r03|CAPMI_LIB=$PWD/ab/lib_r03.so python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_r03.json" \
 "120|b_pk|CAPMI_LIB=$PWD/ab/pk.so python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_pk.json" \
 "120|b_mmpk|python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_mmpk.json" \
 "120|b_r03b|CAPMI_LIB=$PWD/ab/lib_r03.so python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_r03b.json" \
 "120|b_mmpkb|python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_mmpkb.json" \
 "200|c_r03|CAPMI_LIB=$PWD/ab/lib_r03.so python tools/r03/conv_ab.py --arms x3,x3d > gpurun_out/c_r03.md" \
 "200|c_pk|CAPMI_LIB=$PWD/ab/pk.so python tools/r03/conv_ab.py --arms x3,x3d > gpurun_out/c_pk.md" \
 "200|c_mmpk|python tools/r03/conv_ab.py --arms x3,x3d > gpurun_out/c_mmpk.md" \
 "200|c_nosplit|CAPMI_LIB=$PWD/ab/nosplit.so python tools/r03/conv_ab.py --arms x3d > gpurun_out/c_nosplit.md"
