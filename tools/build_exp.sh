# Development only: build an experiment variant of the engine library.
#   bash tools/build_exp.sh NAME "-DMACRO=V ..."  -> foundationdb_amd/lib/libfdb_crc32c_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
D=build/exp_$NAME
mkdir -p $D
for f in foundationdb_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None $* -c $f -o $D/$(basename $f).o &
done
for f in foundationdb_amd/csrc/*.cpp; do
  g++ -O3 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $* -c $f -o $D/$(basename $f).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o foundationdb_amd/lib/libfdb_crc32c_$NAME.so $D/*.o
echo built libfdb_crc32c_$NAME.so
