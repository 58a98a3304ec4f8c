set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -m pytest tests/test_gpu_ba.py -q -x -p no:cacheprovider 2>&1 | tail -2 || exit 1
timeout -k 10 120 python scripts/ba_exp.py 256 384 512 5 2>&1 | grep rep || exit 1
M3S_LIB=lightweight-mast3r-slam_amd/lib/exp/libm3s_stamps.so timeout -k 10 120 python scripts/ba_exp.py 256 384 512 3 2>&1 | grep -v amdgpu.ids
