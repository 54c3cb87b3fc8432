# Development only: build an experiment variant of the engine library.
#   bash tools/build_exp.sh NAME "-DMACRO=V ..."  -> foundationdb_amd/lib/libfdb_crc32c_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
D=build/exp_$NAME
mkdir -p $D
rm -f $D/*.o
for f in foundationdb_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None $* -c $f -o $D/$(basename $f).o &
done
for f in foundationdb_amd/csrc/*.cpp; do
  g++ -O3 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $* -c $f -o $D/$(basename $f).o &
done
wait; for j in $(jobs -p); do :; done
n=$(ls $D/*.o | wc -l); [ "$n" -eq "$(ls foundationdb_amd/csrc/*.hip foundationdb_amd/csrc/*.cpp | wc -l)" ] || { echo "build failed ($n objects)"; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o foundationdb_amd/lib/libfdb_crc32c_$NAME.so $D/*.o
echo built libfdb_crc32c_$NAME.so
