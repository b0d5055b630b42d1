# Build for AMD Instinct MI355X (gfx950). Host code: g++; device code: hipcc --offload-arch=gfx950.
#   make -j8            -> libdllama.so, python extension, dllama, dllama-api
#   make DEBUG=1        -> -O1 -g with host AddressSanitizer/UBSan (device code is not sanitized)
#   make TSAN=1         -> host ThreadSanitizer build (scheduler / API / control plane)
ROCM       ?= /opt/rocm
HIPCC      ?= $(ROCM)/bin/hipcc
CXX        ?= g++
ARCH       ?= gfx950
PKG        := distributed_llama_multiusers_amd
BUILD      := build
PYEXT      := $(shell python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC      := $(shell python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND     := $(shell python3 -c "import pybind11;print(pybind11.get_include())")

OPT        := -O3
SAN        :=
ifeq ($(DEBUG),1)
  OPT := -O1 -g
  SAN := -fsanitize=address,undefined -fno-omit-frame-pointer
endif
ifeq ($(TSAN),1)
  OPT := -O1 -g
  SAN := -fsanitize=thread
endif

HOSTFLAGS  := -std=c++17 $(OPT) -fPIC -march=x86-64-v3 -Wall -Wno-unused-function -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include $(SAN)
HIPFLAGS   := -std=c++17 $(OPT) -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-result -munsafe-fp-atomics $(EXTRA_HIPFLAGS)
# Sanitizer builds instrument the g++-compiled host code (runtime, scheduler, API, TCP, CPU
# backend, tokenizer); the hipcc translation units stay uninstrumented so that one sanitizer
# runtime (gcc's) is linked. Device code is never sanitized on this pool.
LIBLINK    := $(HIPCC) -shared --offload-arch=$(ARCH)
ifneq ($(SAN),)
  LIBLINK  := $(CXX) -shared
endif
LDROCM     := -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrccl

HOST_SRCS  := csrc/core/quant.cpp csrc/core/model_file.cpp csrc/core/plan.cpp csrc/text/tokenizer.cpp \
              csrc/cpu/thread_pool.cpp csrc/cpu/cpu_ops.cpp csrc/cpu/cpu_backend.cpp $(wildcard csrc/net/*.cpp) $(wildcard csrc/runtime/*.cpp)
HIP_SRCS   := csrc/hip/kernels.hip csrc/hip/attn_prefill.hip csrc/hip/sample.hip csrc/hip/tp_check.hip csrc/hip/gemm.hip csrc/hip/gemm_wide.hip csrc/hip/attn_mfma.hip csrc/hip/gemv.hip csrc/hip/gemv_l16.hip csrc/hip/gemv_l32.hip csrc/hip/gemv_l64.hip csrc/hip/attn_block.hip csrc/hip/ffn_block.hip csrc/hip/attn_block_16_16_128.hip csrc/hip/attn_block_16_32_128.hip csrc/hip/attn_block_32_32_128.hip csrc/hip/attn_block_64_32_128.hip csrc/hip/attn_block_64_16_128.hip csrc/hip/attn_block_64_64_128.hip csrc/hip/attn_block_32_64_128.hip csrc/hip/attn_block_64_64_64.hip csrc/hip/engine.cpp csrc/hip/engine_load.cpp csrc/hip/engine_kv.cpp csrc/hip/engine_forward.cpp csrc/hip/engine_bench.cpp csrc/hip/rccl_comm.cpp csrc/hip/sim_comm.cpp csrc/hip/xgmi_comm.cpp csrc/hip/ops.cpp
HOST_OBJS  := $(patsubst csrc/%.cpp,$(BUILD)/obj/%.o,$(HOST_SRCS))
HIP_OBJS   := $(patsubst csrc/%,$(BUILD)/obj/%.o,$(HIP_SRCS))
HDRS       := $(wildcard csrc/*/*.h)

LIB        := $(PKG)/libdllama.so
EXT        := $(PKG)/_C$(PYEXT)
APPS       := $(BUILD)/dllama $(BUILD)/dllama-api

all: $(LIB) $(EXT) $(APPS) $(BUILD)/unit_tests

lib: $(LIB) $(EXT)

$(BUILD)/obj/%.o: csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/obj/hip/%.hip.o: csrc/hip/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/obj/hip/%.cpp.o: csrc/hip/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(HOST_OBJS) $(HIP_OBJS)
	$(LIBLINK) -o $@ $^ $(LDROCM) -lpthread $(SAN) -Wl,-soname,libdllama.so

$(BUILD)/obj/python/bindings.o: csrc/python/bindings.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -I$(PYINC) -I$(PYBIND) -fvisibility=hidden -c $< -o $@

$(EXT): $(BUILD)/obj/python/bindings.o $(LIB)
	$(CXX) -shared -o $@ $< -L$(PKG) -ldllama -Wl,-rpath,'$$ORIGIN' $(LDROCM) $(SAN)

$(BUILD)/obj/apps/%.o: csrc/apps/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/dllama: $(BUILD)/obj/apps/dllama.o $(LIB)
	$(CXX) -o $@ $< -L$(PKG) -ldllama -Wl,-rpath,'$$ORIGIN/../$(PKG)' $(LDROCM) -lpthread $(SAN)

$(BUILD)/dllama-api: $(BUILD)/obj/apps/dllama_api.o $(LIB)
	$(CXX) -o $@ $< -L$(PKG) -ldllama -Wl,-rpath,'$$ORIGIN/../$(PKG)' $(LDROCM) -lpthread $(SAN)

# native unit tests (host code only): build/unit_tests
$(BUILD)/unit_tests: tests/cpp/unit_tests.cpp $(LIB) $(HDRS)
	@mkdir -p $(BUILD)
	$(CXX) $(HOSTFLAGS) -o $@ $< -L$(PKG) -ldllama -Wl,-rpath,'$$ORIGIN/../$(PKG)' $(LDROCM) -lpthread $(SAN)

test-cpp: $(BUILD)/unit_tests
	$(BUILD)/unit_tests

# ring GEMV / attention block instances compile without scratch (inline-asm ring registers are never spilled)
check-isa:
	python3 scripts/check_isa.py

clean:
	rm -rf $(BUILD) $(LIB) $(EXT)

.PHONY: all lib clean test-cpp check-isa
