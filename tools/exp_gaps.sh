# Which host phase leaves the GPU idle at c128 (roctx ranges + kernel trace), then drop the big db.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 env MX_ROCTX=1 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/prof_gaps -o run -- \
  python3 bench.py --path engine --steps 100 --warmup 150 > gpurun_out/prof_gaps.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_gaps.log | tail -1 | cut -c1-300
python tools/gap_regions.py gpurun_out/prof_gaps --min-us 300 | tee gpurun_out/gap_regions.txt
python tools/gap_regions.py gpurun_out/prof_gaps --min-us 50 | tee -a gpurun_out/gap_regions.txt
rm -rf gpurun_out/prof_gaps
