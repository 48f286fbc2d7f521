bash tools/gpu_pmc_fc1.sh r06h pp && bash tools/gpu_pmc_fc1.sh r06h_w4 w4
