# kungfu-amd native build.
#
#   make -j8            host runtime + python binding + launcher binaries + HIP kernels
#   make runtime        host runtime only (no hipcc)
#   make hip            HIP kernel extension only (gfx950)
#
# Outputs (in-tree so they travel with the repo snapshot to the GPU box):
#   kungfu_amd/lib/libkungfu_amd.so       C++ runtime + extern "C" ABI
#   kungfu_amd/_kungfu$(PYEXT)            pybind11 binding of the runtime
#   kungfu_amd/_hip$(PYEXT)               HIP/CDNA4 kernels + RCCL controller (torch extension)
#   bin/kungfu-run, bin/kungfu-config-server, bin/kungfu-rrun, bin/kungfu-distribute, bin/kungfu-test-util,
#   bin/kungfu-bad-worker

# ./configure writes config.mk (build toggles); defaults: trace scopes compiled in,
# HIP kernels + RCCL built, native tests built on demand.
-include config.mk
KUNGFU_ENABLE_TRACE ?= 1
KUNGFU_ENABLE_HIP   ?= 1
PYTHON     ?= python3
CXX        ?= g++
HIPCC      ?= /opt/rocm/bin/hipcc
ARCH       ?= gfx950
BUILD      := build
PYINC      := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
PYEXT      := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
TORCH_DIR  := $(shell $(PYTHON) -c "import os,torch;print(os.path.dirname(torch.__file__))" 2>/dev/null)

CXXFLAGS   := -std=c++17 -O3 -fPIC -Wall -Wextra -Wno-unused-parameter -Icsrc/include -mavx2 -mf16c -pthread $(EXTRA_CXXFLAGS)
ifeq ($(KUNGFU_ENABLE_TRACE),0)
CXXFLAGS   += -DKUNGFU_DISABLE_TRACE
endif
LDFLAGS    := -pthread -ldl $(EXTRA_LDFLAGS)

RT_SRCS    := base plan log monitor transport session http peer capi model_avg scheduler
RT_OBJS    := $(patsubst %,$(BUILD)/rt/%.o,$(RT_SRCS))
RT_LIB     := kungfu_amd/lib/libkungfu_amd.so
PY_MOD     := kungfu_amd/_kungfu$(PYEXT)

LAUNCH_SRCS := runner job configserver_main flags
LAUNCH_OBJS := $(patsubst %,$(BUILD)/launcher/%.o,$(LAUNCH_SRCS))
BINS       := bin/kungfu-run bin/kungfu-config-server bin/kungfu-rrun bin/kungfu-distribute bin/kungfu-test-util \
              bin/kungfu-bad-worker

HIP_SRCS   := $(wildcard csrc/kernels/*.hip)
HIP_OBJS   := $(patsubst csrc/kernels/%.hip,$(BUILD)/hip/%.o,$(HIP_SRCS))
HIP_BIND   := $(BUILD)/hip/bindings.o
HIP_MOD    := kungfu_amd/_hip$(PYEXT)
HIPFLAGS   := -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) -Icsrc/include -D__HIP_PLATFORM_AMD__ \
              -ffp-contract=fast -munsafe-fp-atomics -Wno-unused-result $(EXTRA_HIPFLAGS)
TORCH_INC  := -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -I$(PYINC) -I$(PYBIND_INC)
TORCH_LIBS := -L$(TORCH_DIR)/lib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python \
              -Wl,-rpath,$(TORCH_DIR)/lib

.PHONY: all runtime hip launcher clean
ifeq ($(KUNGFU_ENABLE_HIP),0)
all: runtime launcher   # host-only build: no hipcc, no RCCL (CPU / gloo-style training)
else
all: runtime launcher hip
endif
runtime: $(RT_LIB) $(PY_MOD)
launcher: $(BINS)
hip: $(HIP_MOD)

$(BUILD)/rt/%.o: csrc/runtime/%.cpp $(wildcard csrc/include/kungfu/*.hpp csrc/include/kungfu/*.h)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(RT_LIB): $(RT_OBJS)
	@mkdir -p $(dir $@)
	$(CXX) -shared -o $@ $^ $(LDFLAGS) -Wl,-soname,libkungfu_amd.so

$(BUILD)/rt/pybind.o: csrc/runtime/pybind.cpp $(wildcard csrc/include/kungfu/*.hpp)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(PYINC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(PY_MOD): $(BUILD)/rt/pybind.o $(RT_LIB)
	$(CXX) -shared -o $@ $< -Lkungfu_amd/lib -lkungfu_amd -Wl,-rpath,'$$ORIGIN/lib' $(LDFLAGS)

$(BUILD)/launcher/%.o: csrc/launcher/%.cpp $(wildcard csrc/include/kungfu/*.hpp csrc/launcher/*.hpp)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -Icsrc/launcher -c $< -o $@

bin/kungfu-run: $(BUILD)/launcher/kungfu_run.o $(LAUNCH_OBJS) $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

bin/kungfu-config-server: $(BUILD)/launcher/config_server_bin.o $(LAUNCH_OBJS) $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

bin/kungfu-rrun: $(BUILD)/launcher/rrun.o $(LAUNCH_OBJS) $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

bin/kungfu-distribute: $(BUILD)/launcher/distribute.o $(LAUNCH_OBJS) $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

bin/kungfu-test-util: $(BUILD)/launcher/test_util.o $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

bin/kungfu-bad-worker: $(BUILD)/launcher/bad_worker.o $(RT_OBJS)
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LDFLAGS)

$(BUILD)/hip/%.o: csrc/kernels/%.hip $(wildcard csrc/kernels/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(HIP_BIND): csrc/kernels/bindings.cpp $(wildcard csrc/kernels/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(TORCH_INC) -DTORCH_EXTENSION_NAME=_hip -DUSE_ROCM -fvisibility=hidden -c $< -o $@

$(HIP_MOD): $(HIP_OBJS) $(HIP_BIND)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ $(TORCH_LIBS) -lrccl -L/opt/rocm/lib

clean:
	rm -rf $(BUILD) $(RT_LIB) $(PY_MOD) $(HIP_MOD) $(BINS)

# ---- native tests (host only; sanitizer builds for race / memory checks) ----
ifeq ($(KUNGFU_BUILD_TESTS),1)
all: build/native_test build/native_test_asan build/native_test_tsan
endif
NT_SRCS := tests/native/test_runtime.cpp $(patsubst %,csrc/runtime/%.cpp,$(RT_SRCS))
.PHONY: native-test native-test-asan native-test-tsan
build/native_test: $(NT_SRCS) $(wildcard csrc/include/kungfu/*.hpp)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -g -o $@ $(NT_SRCS) $(LDFLAGS)
build/native_test_asan: $(NT_SRCS) $(wildcard csrc/include/kungfu/*.hpp)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -o $@ $(NT_SRCS) $(LDFLAGS)
build/native_test_tsan: $(NT_SRCS) $(wildcard csrc/include/kungfu/*.hpp)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -O1 -g -fsanitize=thread -o $@ $(NT_SRCS) $(LDFLAGS)
native-test: build/native_test
	./build/native_test
native-test-asan: build/native_test_asan
	./build/native_test_asan 42000
native-test-tsan: build/native_test_tsan
	TSAN_OPTIONS=halt_on_error=1 ./build/native_test_tsan 43000
