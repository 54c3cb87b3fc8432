# Build the MI355X CRC-32C engine (C-ABI shared library) and the test oracle.
#   make            -> foundationdb_amd/lib/libfdb_crc32c.so + oracle libs
# Device code: hipcc for gfx950 only.  Host code: g++.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
JOBS ?= 8

CSRC := foundationdb_amd/csrc
OBJ := build/obj
LIB := foundationdb_amd/lib/libfdb_crc32c.so
# bounds-checked build for kernel debugging (defined before `all`: prerequisites
# are expanded when a rule is read)
DBG_LIB := foundationdb_amd/lib/libfdb_crc32c_debug.so

HIP_SRCS := $(wildcard $(CSRC)/*.hip)
CPP_SRCS := $(wildcard $(CSRC)/*.cpp)
HDRS := $(wildcard $(CSRC)/*.h) $(wildcard include/*.h)
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJ)/%.hip.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst $(CSRC)/%.cpp,$(OBJ)/%.cpp.o,$(CPP_SRCS))

HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result
CXXFLAGS := -O3 -fPIC -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include

# test/bench utilities (synthetic data in HBM, LDS poisoning): their own
# library, never linked into the product
TU_LIB := foundationdb_amd/lib/libfdb_crc32c_testutil.so
TU_SRCS := $(wildcard foundationdb_amd/testutil/*.hip)

all: $(LIB) $(TU_LIB) $(DBG_LIB) oracle

$(TU_LIB): $(TU_SRCS) foundationdb_amd/testutil/fdb_crc32c_testutil.h
	@mkdir -p $(dir $(TU_LIB))
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(TU_SRCS)

# the page kernels' grab requests must stay single-lane atomics whose return is
# awaited only where it is used (the atomic optimizer's wave reduction reads it
# back at once, which stalls on every data load in flight)
$(OBJ)/crc32c_kernels.hip.o $(OBJ)/crc32c_extent.hip.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None

$(OBJ)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -C oracle

# bounds-checked build for kernel debugging (foundationdb_amd/lib/libfdb_crc32c_debug.so)
# (built by default: the GPU suite replays route batches against it)
DBG_OBJS := $(patsubst $(CSRC)/%.hip,build/dbg/%.hip.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,build/dbg/%.cpp.o,$(CPP_SRCS))
build/dbg/crc32c_kernels.hip.o build/dbg/crc32c_extent.hip.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None
build/dbg/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build/dbg
	$(HIPCC) $(HIPFLAGS) -DFDBCRC_DEBUG -c $< -o $@
build/dbg/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build/dbg
	$(CXX) $(CXXFLAGS) -DFDBCRC_DEBUG -c $< -o $@
$(DBG_LIB): $(DBG_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^
debug: $(DBG_LIB)

# ASan + UBSan build of the host code (reference: cmake/ConfigureCompiler.cmake:5-12):
# every .cpp instrumented, the device objects as in the product; load it with
#   LD_PRELOAD=$$(g++ -print-file-name=libasan.so) FDBCRC_LIB=$(ASAN_LIB) python ...
# (tools/run_asan.sh runs the non-GPU suite that way).
ASAN_LIB := foundationdb_amd/lib/libfdb_crc32c_asan.so
SANFLAGS := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
ASAN_OBJS := $(patsubst $(CSRC)/%.cpp,build/asan/%.cpp.o,$(CPP_SRCS))
build/asan/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build/asan
	$(CXX) $(CXXFLAGS) $(SANFLAGS) -c $< -o $@
$(ASAN_LIB): $(HIP_OBJS) $(ASAN_OBJS)
	$(CXX) -shared $(SANFLAGS) -o $@ $^ -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib
asan: $(ASAN_LIB)

clean:
	rm -rf build $(LIB) $(TU_LIB) $(ASAN_LIB) $(DBG_LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean debug asan
