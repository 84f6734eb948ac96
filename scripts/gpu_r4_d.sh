# round 4, GPU call D: steady-state video job (30k frames per job from a looped 3000-frame npy, host busy
# time per stage of the requester and both workers), both data planes, 3 interleaved runs each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/d || exit 1
timeout -k 10 900 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both \
  > gpurun_out/d/bench_video_30k.log 2>&1
echo "rc=$?" >> gpurun_out/d/bench_video_30k.log
