# vision session, then the video job benchmark (one box acquisition)
bash scripts/gpu_r3_vision.sh && bash scripts/gpu_r3_video.sh
