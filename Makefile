# Builds the in-tree C-ABI library dstagnn_drought_amd/libdstagnn.so for gfx950 (MI355X).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC := $(wildcard dstagnn_drought_amd/csrc/*.hip)
OBJ := $(patsubst dstagnn_drought_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := dstagnn_drought_amd/libdstagnn.so
# host build of the EMD solver for the CPU tests only (the package never loads it)
EMD_HOST := tests/native/libemd_host.so
# the PyTorch-ROCm operator library (TORCH_LIBRARY(dstagnn, ...)) over libdstagnn.so
EXT := dstagnn_drought_amd/_C.so
PY ?= python3
TORCH_DIR := $(shell $(PY) -c "import os, torch; print(os.path.dirname(torch.__file__))" 2>/dev/null)
TORCH_ABI := $(shell $(PY) -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))" 2>/dev/null)
EXT_FLAGS := -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$(TORCH_ABI) \
	-I/opt/rocm/include -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -Wno-unused-result
EXT_LIBS := -L$(TORCH_DIR)/lib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip \
	-Ldstagnn_drought_amd -ldstagnn -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib

# deliberately racy variant for the race-probe self-check (tests/test_gpu_knobs.py): the same
# objects with block.o rebuilt under -DDSTAGNN_RACEBUG_NOFORK (never loaded by the package)
RACEBUG := abtest/racebug/libdstagnn.so

# hipcc-built host program driving the block through the C-ABI alone (tests/test_gpu_native_abi.py)
ABI_TEST := tests/native/block_abi_test

all: $(LIB) $(EXT) $(EMD_HOST) tools/fetch_calib $(RACEBUG) $(ABI_TEST)

racebug: $(RACEBUG)

build/racebug/block.o: dstagnn_drought_amd/csrc/block.hip dstagnn_drought_amd/csrc/*.hpp include/dstagnn.h
	@mkdir -p build/racebug
	$(HIPCC) $(CXXFLAGS) -DDSTAGNN_RACEBUG_NOFORK -c $< -o $@

$(RACEBUG): $(filter-out build/block.o,$(OBJ)) build/racebug/block.o
	@mkdir -p abtest/racebug
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^

# phase-timing variant of the fused kernels (-DDSTAGNN_TF_TIMING: per-phase wall-clock printf from
# workgroups 0 and 100), loaded by LD_LIBRARY_PATH=abtest/tftime; not part of `all`
TFTIME := abtest/tftime/libdstagnn.so
TF_SRC := tat_fused gtu_fused sat_fused
tftime: $(TFTIME)

build/tftime/%.o: dstagnn_drought_amd/csrc/%.hip dstagnn_drought_amd/csrc/*.hpp include/dstagnn.h
	@mkdir -p build/tftime
	$(HIPCC) $(CXXFLAGS) -DDSTAGNN_TF_TIMING -c $< -o $@

$(TFTIME): $(filter-out $(patsubst %,build/%.o,$(TF_SRC)),$(OBJ)) $(patsubst %,build/tftime/%.o,$(TF_SRC))
	@mkdir -p abtest/tftime
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^

# FETCH_SIZE / WRITE_SIZE width calibration (tools/pmc_step.sh)
tools/fetch_calib: tools/fetch_calib.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) $< -o $@

$(EXT): dstagnn_drought_amd/csrc/torch_ops.cpp include/dstagnn.h $(LIB)
	@mkdir -p build
	$(HIPCC) $(EXT_FLAGS) -x c++ -c $< -o build/torch_ops.o
	$(HIPCC) -shared -o $@ build/torch_ops.o $(EXT_LIBS)

$(ABI_TEST): tests/native/block_abi_main.cpp include/dstagnn.h $(LIB)
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ $< -Ldstagnn_drought_amd -ldstagnn -Wl,-rpath,'$$ORIGIN/../../dstagnn_drought_amd'

$(EMD_HOST): tests/native/emd_host.cpp dstagnn_drought_amd/csrc/emd_simplex.hpp
	g++ -O2 -std=c++17 -fPIC -shared -Wall -o $@ $<

build/%.o: dstagnn_drought_amd/csrc/%.hip dstagnn_drought_amd/csrc/*.hpp include/dstagnn.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB) $(EXT) $(EMD_HOST) $(ABI_TEST) tools/fetch_calib abtest/racebug abtest/tftime

.PHONY: all clean racebug tftime
