#!/bin/bash
# PMC passes on the default-init and the opaque-sphere scene
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/pmc_r2.sh r2r_def > gpurun_out/r2r_def.log 2>&1 || { tail -20 gpurun_out/r2r_def.log; exit 1; }
bash tools/pmc_r2.sh r2r_surf --scene surface > gpurun_out/r2r_surf.log 2>&1 || { tail -20 gpurun_out/r2r_surf.log; exit 1; }
grep -E "k_final|k_sgrid_box4|k_prop_sigma" gpurun_out/pmc_r2r_def/table.txt | cut -c1-900
echo ---
grep -E "k_final|k_sgrid_box4|k_prop_sigma" gpurun_out/pmc_r2r_surf/table.txt | cut -c1-900
