bash tools/gpu_r3r.sh && bash tools/gpu_r3final.sh
