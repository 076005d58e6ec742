bash tools/gpu_check.sh r04f
