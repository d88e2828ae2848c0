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

HOST_SRC := $(ROOT)stem_kernel_amd/csrc/host/synth.cpp $(ROOT)stem_kernel_amd/csrc/host/example_build.cpp \
            $(ROOT)stem_kernel_amd/csrc/host/readers.cpp $(ROOT)stem_kernel_amd/csrc/host/shard.cpp \
            $(ROOT)stem_kernel_amd/csrc/host/svm_predict.cpp
API_SRC := $(ROOT)stem_kernel_amd/csrc/sk_api.cpp
HIP_SRC := $(ROOT)stem_kernel_amd/csrc/kernels/dag_stem.hip $(ROOT)stem_kernel_amd/csrc/kernels/profile_string.hip \
           $(ROOT)stem_kernel_amd/csrc/kernels/bpla.hip $(ROOT)stem_kernel_amd/csrc/kernels/stem4d.hip \
           $(ROOT)stem_kernel_amd/csrc/kernels/phmm.hip $(ROOT)stem_kernel_amd/csrc/kernels/bpla_grad.hip \
           $(ROOT)stem_kernel_amd/csrc/kernels/dag_stem_big.hip $(ROOT)stem_kernel_amd/csrc/kernels/fold.hip
HDRS := $(wildcard $(ROOT)stem_kernel_amd/csrc/*/*.h) $(ROOT)include/stem_kernel.h $(ROOT)stem_kernel_amd/csrc/ribosum85_60.inc

HOST_OBJ := $(patsubst $(ROOT)stem_kernel_amd/csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC) $(API_SRC))
HIP_OBJ := $(patsubst $(ROOT)stem_kernel_amd/csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))

all: lib cli oracle exp

lib: $(LIB)

# the reference's stem_kernel_lite CLI over the engine (host C++, links the library)
CLI := $(ROOT)stem_kernel_amd/bin/stem_kernel_lite
cli: $(CLI)
$(CLI): $(ROOT)stem_kernel_amd/csrc/cli/stem_kernel_lite.cpp $(ROOT)include/stem_kernel_compat.hpp $(ROOT)include/stem_kernel.h $(LIB)
	@mkdir -p $(dir $@)
	g++ -O2 -std=c++17 -Wall -Wextra -I$(ROOT)include $< -L$(ROOT)stem_kernel_amd -lstem_kernel_amd -lz -ldl \
	  -Wl,-rpath,'$$ORIGIN/..' -o $@

$(BUILD)/%.o: $(ROOT)stem_kernel_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(BUILD)/%.o: $(ROOT)stem_kernel_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# the PairHMM's log-space sums must round like the host restatement
$(BUILD)/kernels/phmm.o: HIPFLAGS += -ffp-contract=off
$(BUILD)/kernels/bpla_grad.o: HIPFLAGS += -ffp-contract=off
# the synthetic fold's AVX2 clone and baseline must round alike (no FMA)
$(BUILD)/host/synth.o: CXXFLAGS += -ffp-contract=off

$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C $(ROOT)oracle

clean:
	rm -rf $(BUILD) $(LIB) $(CLI)
	$(MAKE) -C $(ROOT)oracle clean

.PHONY: all lib cli oracle clean

# diagnostic build with in-kernel phase stamps (never the shipped library)
STAMPS_LIB := $(ROOT)build/libstem_kernel_amd_stamps.so
stamps:
	@mkdir -p $(BUILD)/stamps
	$(HIPCC) $(HIPFLAGS) -DSK_STAMPS -x hip -c $(ROOT)stem_kernel_amd/csrc/kernels/dag_stem.hip -o $(BUILD)/stamps/dag_stem.o
	$(HIPCC) $(CXXFLAGS) -DSK_STAMPS -D__HIP_PLATFORM_AMD__ -c $(API_SRC) -o $(BUILD)/stamps/sk_api.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(STAMPS_LIB) $(BUILD)/host/synth.o $(BUILD)/host/example_build.o $(BUILD)/host/readers.o $(BUILD)/host/shard.o $(BUILD)/host/svm_predict.o $(BUILD)/stamps/sk_api.o $(BUILD)/stamps/dag_stem.o $(BUILD)/kernels/profile_string.o $(BUILD)/kernels/bpla.o $(BUILD)/kernels/stem4d.o $(BUILD)/kernels/phmm.o $(BUILD)/kernels/bpla_grad.o $(BUILD)/kernels/dag_stem_big.o $(BUILD)/kernels/fold.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: stamps

# experiment build: make variant NAME=x DEFS="-DSK_PW=3 [-DSK_STAMPS]" -> build/libsk_x.so
variant:
	@mkdir -p $(BUILD)/var/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -x hip -c $(ROOT)stem_kernel_amd/csrc/kernels/dag_stem.hip -o $(BUILD)/var/$(NAME)/dag_stem.o
	$(HIPCC) $(CXXFLAGS) $(DEFS) -D__HIP_PLATFORM_AMD__ -c $(API_SRC) -o $(BUILD)/var/$(NAME)/sk_api.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(BUILD)/libsk_$(NAME).so $(BUILD)/host/synth.o $(BUILD)/host/example_build.o $(BUILD)/host/readers.o $(BUILD)/host/shard.o $(BUILD)/host/svm_predict.o $(BUILD)/var/$(NAME)/sk_api.o $(BUILD)/var/$(NAME)/dag_stem.o $(BUILD)/kernels/profile_string.o $(BUILD)/kernels/bpla.o $(BUILD)/kernels/stem4d.o $(BUILD)/kernels/phmm.o $(BUILD)/kernels/bpla_grad.o $(BUILD)/kernels/dag_stem_big.o $(BUILD)/kernels/fold.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: variant

# fold kernel experiment build: make variantf NAME=x DEFS="-DSK_FOLD_TIMING" -> build/libsk_x.so
variantf:
	@mkdir -p $(BUILD)/var/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -x hip -c $(ROOT)stem_kernel_amd/csrc/kernels/fold.hip -o $(BUILD)/var/$(NAME)/fold.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(BUILD)/libsk_$(NAME).so $(BUILD)/host/synth.o $(BUILD)/host/example_build.o $(BUILD)/host/readers.o $(BUILD)/host/shard.o $(BUILD)/host/svm_predict.o $(BUILD)/sk_api.o $(BUILD)/kernels/dag_stem.o $(BUILD)/kernels/profile_string.o $(BUILD)/kernels/bpla.o $(BUILD)/kernels/stem4d.o $(BUILD)/kernels/phmm.o $(BUILD)/kernels/bpla_grad.o $(BUILD)/kernels/dag_stem_big.o $(BUILD)/var/$(NAME)/fold.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: variantf

# 4-D kernel experiment build: make variant4 NAME=x DEFS="-DSK4_MINB=4" -> build/libsk_x.so
variant4:
	@mkdir -p $(BUILD)/var/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -x hip -c $(ROOT)stem_kernel_amd/csrc/kernels/stem4d.hip -o $(BUILD)/var/$(NAME)/stem4d.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(BUILD)/libsk_$(NAME).so $(BUILD)/host/synth.o $(BUILD)/host/example_build.o $(BUILD)/host/readers.o $(BUILD)/host/shard.o $(BUILD)/host/svm_predict.o $(BUILD)/sk_api.o $(BUILD)/kernels/dag_stem.o $(BUILD)/kernels/profile_string.o $(BUILD)/kernels/bpla.o $(BUILD)/var/$(NAME)/stem4d.o $(BUILD)/kernels/phmm.o $(BUILD)/kernels/bpla_grad.o $(BUILD)/kernels/dag_stem_big.o $(BUILD)/kernels/fold.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: variant4

# experiments build: the shipped sources with the A/B switches compiled in
# (SK_KNOB reads the environment; sk_experiments() = 1) -> build/libstem_kernel_amd_exp.so,
# loaded by the GPU tests that compare kernel variants (tests/explib.py)
EXP_LIB := $(ROOT)build/libstem_kernel_amd_exp.so
EXP_OBJ := $(patsubst $(ROOT)stem_kernel_amd/csrc/%.cpp,$(BUILD)/exp/%.o,$(HOST_SRC) $(API_SRC))
exp: $(EXP_LIB)
$(BUILD)/exp/%.o: $(ROOT)stem_kernel_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -DSK_EXPERIMENTS -D__HIP_PLATFORM_AMD__ -c $< -o $@
$(BUILD)/exp/host/synth.o: CXXFLAGS += -ffp-contract=off
$(EXP_LIB): $(EXP_OBJ) $(HIP_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: exp
