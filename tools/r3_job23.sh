set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
for B in 16 32 64 128 256; do timeout -k 10 120 python tools/time_sampler.py --B $B 2>&1 | grep -v amdgpu.ids || exit 1; done
