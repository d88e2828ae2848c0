# Build of the MI355X stem-kernel engine (gfx950) and the test oracle.
#   make            -> stem_kernel_amd/libstem_kernel_amd.so + oracle
#   make lib        -> product library only
#   make oracle     -> oracle/liboracle.so (+ oracle/_ref when /root/reference exists)
ROOT := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I$(ROOT)include -I$(ROOT)stem_kernel_amd/csrc
HIPFLAGS := $(CXXFLAGS) --offload-arch=$(ARCH) -munsafe-fp-atomics
BUILD := $(ROOT)build
LIB := $(ROOT)stem_kernel_amd/libstem_kernel_amd.so

HOST_SRC := $(ROOT)stem_kernel_amd/csrc/host/synth.cpp $(ROOT)stem_kernel_amd/csrc/host/example_build.cpp
API_SRC := $(ROOT)stem_kernel_amd/csrc/sk_api.cpp
HIP_SRC := $(ROOT)stem_kernel_amd/csrc/kernels/dag_stem.hip $(ROOT)stem_kernel_amd/csrc/kernels/profile_string.hip
HDRS := $(wildcard $(ROOT)stem_kernel_amd/csrc/*/*.h) $(ROOT)include/stem_kernel.h $(ROOT)stem_kernel_amd/csrc/ribosum85_60.inc

HOST_OBJ := $(patsubst $(ROOT)stem_kernel_amd/csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC) $(API_SRC))
HIP_OBJ := $(patsubst $(ROOT)stem_kernel_amd/csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))

all: lib oracle

lib: $(LIB)

$(BUILD)/%.o: $(ROOT)stem_kernel_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(BUILD)/%.o: $(ROOT)stem_kernel_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C $(ROOT)oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -C $(ROOT)oracle clean

.PHONY: all lib oracle clean
