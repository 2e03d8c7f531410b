set -e
O=gpurun_out/v1x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden_big.py tests/test_gpu_exact_lookahead.py tests/test_gpu_configs.py tests/test_fuzz.py -m gpu > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/prof_exact_c3.py --version 1 > $O/new_v1_$i.json 2>&1
  PSS_LIB=build/ab/v1old/libpss.so timeout -k 10 200 python tools/prof_exact_c3.py --version 1 > $O/old_v1_$i.json 2>&1
  timeout -k 10 200 python tools/prof_exact_c3.py --version 1 --cfg c2 --epochs 20 > $O/new_v1c2_$i.json 2>&1
  PSS_LIB=build/ab/v1old/libpss.so timeout -k 10 200 python tools/prof_exact_c3.py --version 1 --cfg c2 --epochs 20 > $O/old_v1c2_$i.json 2>&1
  timeout -k 10 200 python tools/prof_exact_c3.py > $O/new_v2_$i.json 2>&1
done
echo ok
