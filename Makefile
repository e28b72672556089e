# Builds the in-tree C-ABI library dstagnn_drought_amd/libdstagnn.so for gfx950 (MI355X).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC := $(wildcard dstagnn_drought_amd/csrc/*.hip)
OBJ := $(patsubst dstagnn_drought_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := dstagnn_drought_amd/libdstagnn.so
# host build of the EMD solver for the CPU tests only (the package never loads it)
EMD_HOST := tests/native/libemd_host.so

all: $(LIB) $(EMD_HOST)

$(EMD_HOST): tests/native/emd_host.cpp dstagnn_drought_amd/csrc/emd_simplex.hpp
	g++ -O2 -std=c++17 -fPIC -shared -Wall -o $@ $<

build/%.o: dstagnn_drought_amd/csrc/%.hip dstagnn_drought_amd/csrc/*.hpp include/dstagnn.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB) $(EMD_HOST)

.PHONY: all clean
