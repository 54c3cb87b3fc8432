# Per-kernel register, spill, occupancy and LDS figures of the product
# kernels (-Rpass-analysis=kernel-resource-usage), one block per kernel:
#   bash tools/resource_usage.sh > profiles/roundN/resource_usage.txt
cd "$(dirname "$0")/.."
for f in foundationdb_amd/csrc/*.hip; do
  echo "=== $(basename $f)"
  extra=""
  case $f in *crc32c_kernels.hip|*crc32c_extent.hip) extra="-mllvm -amdgpu-atomic-optimizer-strategy=None";; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $extra -Rpass-analysis=kernel-resource-usage -c $f -o /tmp/ru.o 2>&1 |
    grep -E "remark: +(Function Name|TotalSGPRs|VGPRs|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size)" |
    sed -E 's/.*remark: +//; s/ \[-Rpass-analysis=kernel-resource-usage\]//'
done
