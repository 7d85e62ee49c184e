set -o pipefail
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
echo "== ship"; AB_VAR=ANOMOD_BUCKET_AVG AB_VALS=1400 timeout -k 10 200 python3 scripts/time_env_ab.py 27 3 | tail -1 || exit 1
echo "== w1k"; ANOMOD_LIB=$PWD/$V/libanomod_w1k.so AB_VAR=ANOMOD_BUCKET_AVG AB_VALS=1400,2600 timeout -k 10 200 python3 scripts/time_env_ab.py 27 3 | tail -1 || exit 1
ANOMOD_LIB=$PWD/$V/libanomod_w1k.so ANOMOD_BUCKET_AVG=2600 timeout -k 10 200 python3 -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group.py | tail -1 || exit 2
