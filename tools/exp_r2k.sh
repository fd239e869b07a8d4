# Stable Video Diffusion (SVD 14 frames, 1024x576) timing, Whisper-base refresh (BASELINE config #4),
# and the c128 GPU idle-gap picture with roctx step ranges.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u tools/bench_svd.py --model svd --width 1024 --height 576 --steps 4 > gpurun_out/k_svd.json 2> gpurun_out/k_svd.err || { tail -20 gpurun_out/k_svd.err; exit 1; }
tail -1 gpurun_out/k_svd.json
timeout -k 10 300 python -u tools/bench_whisper.py --model whisper-base --seconds 120 --tokens 128 > gpurun_out/k_whisper.jsonl 2> gpurun_out/k_whisper.err || { tail -20 gpurun_out/k_whisper.err; exit 1; }
tail -2 gpurun_out/k_whisper.jsonl
timeout -k 10 400 env MX_ROCTX=1 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/prof_gaps2 -o run -- python3 bench.py --path engine --steps 100 --warmup 150 > gpurun_out/prof_gaps2.log 2>&1 || { tail -20 gpurun_out/prof_gaps2.log; exit 1; }
grep '^{' gpurun_out/prof_gaps2.log | tail -1 | cut -c1-200
python tools/trace_gaps.py gpurun_out/prof_gaps2 > gpurun_out/k_gaps.txt 2>&1 || true
head -12 gpurun_out/k_gaps.txt
python tools/gap_regions.py gpurun_out/prof_gaps2 --min-us 50 > gpurun_out/k_gap_regions.txt 2>&1 || true
head -20 gpurun_out/k_gap_regions.txt
rm -rf gpurun_out/prof_gaps2
