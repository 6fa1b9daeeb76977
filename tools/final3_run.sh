bash tools/final_check.sh gpurun_out/r06_final3 core && bash tools/final_check.sh gpurun_out/r06_final3_scale scale
