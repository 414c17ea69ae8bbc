bash scripts/r4/gpu_d.sh && bash scripts/r4/gpu_e.sh
