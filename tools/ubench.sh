set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w -o build/ubench_valu tools/ubench_valu.hip
timeout -k 10 120 ./build/ubench_valu | tee gpurun_out/ubench_valu.log
