# Build for MI355X (gfx950).  Host C++ with g++ (OpenMP via libgomp, the same
# runtime PyTorch ships), device code with hipcc --offload-arch=gfx950.
#   make            → python extension + CLI apps (bin/pe_hip, bin/pe_cpu, bin/pe_launch)
#   make cpu        → CPU-only pieces
#   make clean
ROCM      ?= /opt/rocm
ARCH      ?= gfx950
PYTHON    ?= python3
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
PKG       := poisson_ellipse_openmp_mpi_cuda_amd
BUILD     := build
BIN       := bin

PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
EXT_SUF   := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

COMMON    := -O3 -std=c++17 -fPIC -Wall -Wno-unknown-pragmas -Icsrc/include
CXXFLAGS  += $(COMMON) -fopenmp -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
# Device code: exact IEEE fp64 (no contraction) so the device operator
# matches the CPU oracle operation-for-operation; code object v5 for the
# ROCm 7.0 runtime bundled with PyTorch.
HIPFLAGS  += $(COMMON) --offload-arch=$(ARCH) -ffp-contract=off -mcode-object-version=5 \
             -fno-gpu-rdc -munsafe-fp-atomics
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -lgomp -lpthread -Wl,-rpath,$(ROCM)/lib

CORE_SRC  := csrc/core/decomp.cpp csrc/core/thread_comm.cpp csrc/core/report.cpp csrc/cpu/pcg_cpu.cpp
HOST_SRC  := csrc/hip/device_solver.cpp csrc/hip/item_layout.cpp csrc/hip/placement.cpp csrc/hip/checkpoint.cpp csrc/hip/halo_path.cpp csrc/hip/rccl_comm.cpp csrc/hip/p2p_comm.cpp csrc/hip/runtime.cpp csrc/core/row_classes.cpp
HIP_SRC   := csrc/hip/kernels.hip csrc/hip/fused.hip csrc/hip/fused2.hip csrc/hip/fused3.hip csrc/hip/resident.hip csrc/hip/p2p.hip
BIND_SRC  := csrc/bind/module.cpp

CORE_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(CORE_SRC))
HOST_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC))
HIP_OBJ   := $(patsubst csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))
BIND_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(BIND_SRC))
HEADERS   := $(wildcard csrc/include/pe/*.hpp) $(wildcard csrc/hip/*.hpp) csrc/apps/args.hpp

EXT       := $(PKG)/_native$(EXT_SUF)

.PHONY: all cpu clean asan tsan
all: $(EXT) $(BIN)/pe_hip $(BIN)/pe_cpu $(BIN)/pe_launch
cpu: $(BIN)/pe_cpu

$(BUILD)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/hip/%.o: csrc/hip/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/bind/module.o: csrc/bind/module.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(EXT): $(CORE_OBJ) $(HOST_OBJ) $(HIP_OBJ) $(BIND_OBJ)
	$(CXX) -shared -o $@ $^ $(LDLIBS)

$(BIN)/pe_cpu: $(BUILD)/apps/pe_cpu.o $(CORE_OBJ)
	@mkdir -p $(BIN)
	$(CXX) -o $@ $^ -lgomp -lpthread

$(BIN)/pe_hip: $(BUILD)/apps/pe_hip.o $(CORE_OBJ) $(HOST_OBJ) $(HIP_OBJ)
	@mkdir -p $(BIN)
	$(CXX) -o $@ $^ $(LDLIBS)

$(BIN)/pe_launch: $(BUILD)/apps/pe_launch.o
	@mkdir -p $(BIN)
	$(CXX) -o $@ $^ -lpthread

# Host sanitizer builds of the CPU solver (the GPU pool has no device
# ASan / XNACK): AddressSanitizer + UBSan, and ThreadSanitizer for the
# thread-rank transport (run with --threads 1: libgomp is not TSan-built).
SAN_SRC   := $(CORE_SRC) csrc/apps/pe_cpu.cpp
asan: $(BIN)/pe_cpu_asan
tsan: $(BIN)/pe_cpu_tsan
$(BIN)/pe_cpu_asan: $(SAN_SRC) $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) -O1 -g -std=c++17 -Wall -Wno-unknown-pragmas -Icsrc/include -fopenmp -fno-omit-frame-pointer \
	  -fsanitize=address,undefined -fno-sanitize-recover=undefined $(SAN_SRC) -o $@ -lpthread
$(BIN)/pe_cpu_tsan: $(SAN_SRC) $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) -O1 -g -std=c++17 -Wall -Wno-unknown-pragmas -Icsrc/include -fopenmp -fsanitize=thread $(SAN_SRC) \
	  -o $@ -lpthread

clean:
	rm -rf $(BUILD) $(BIN) $(EXT)
