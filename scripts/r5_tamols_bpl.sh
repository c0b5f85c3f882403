set -e
for v in bpl16 bpl4 bpl8 bpl32 bpl16; do
  echo "== $v"
  SRBD_LIB_PATH=$PWD/quadruped-pympc-tamols_amd/variants/lib_$v.so timeout -k 10 100 python -u scripts/tamols_probe.py
  SRBD_LIB_PATH=$PWD/quadruped-pympc-tamols_amd/variants/lib_$v.so timeout -k 10 100 python -u scripts/c4_split.py 2000
done
SRBD_LIB_PATH=$PWD/quadruped-pympc-tamols_amd/variants/lib_bpl4.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tamols.py tests/test_gpu_c4_pipeline.py tests/test_gpu_terrain.py 2>&1 | tail -2
SRBD_LIB_PATH=$PWD/quadruped-pympc-tamols_amd/variants/lib_bpl32.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tamols.py tests/test_gpu_c4_pipeline.py tests/test_gpu_terrain.py 2>&1 | tail -2
