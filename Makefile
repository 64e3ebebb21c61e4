# Native build for bitcoincashplus_amd.
#   make            -> core static lib, HIP kernels (gfx950), Python extension, node binaries
#   make pyext      -> only the Python extension
#   make clean
# CPU code is built with g++ (C++17); HIP kernels with hipcc --offload-arch=gfx950.
# Everything lands in-tree: build/ for objects, bitcoincashplus_amd/_bcpnative*.so, bin/.

ROCM       ?= /opt/rocm
HIPCC      ?= $(ROCM)/bin/hipcc
CXX        ?= g++
PYTHON     ?= python3
GPU_ARCH   ?= gfx950
OPT        ?= -O2

PY_INC     := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
PY_EXT     := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

CXXFLAGS   := -std=c++17 $(OPT) -g1 -fPIC -Wall -Wno-unused-function -Wno-sign-compare -Icsrc -pthread
HIPFLAGS   := -std=c++17 $(OPT) -fPIC --offload-arch=$(GPU_ARCH) -Icsrc -munsafe-fp-atomics \
              -Wno-unused-result -Wno-unused-variable -Wno-pass-failed
LDLIBS     := -L$(ROCM)/lib -lamdhip64 -lcrypto -pthread -ldl -Wl,-rpath,$(ROCM)/lib
# hardening of every linked binary and library (contrib/devtools/security-check.py: PIE, NX,
# full RELRO, stack canary; executables get PIE and the canary from the toolchain defaults)
HARDEN_LD  := -Wl,-z,relro,-z,now,-z,noexecstack

CORE_SRCS  := $(wildcard csrc/crypto/*.cpp csrc/primitives/*.cpp csrc/consensus/*.cpp \
                csrc/script/*.cpp csrc/secp256k1/*.cpp csrc/util/*.cpp csrc/node/*.cpp \
                csrc/rpc/*.cpp csrc/net/*.cpp csrc/wallet/*.cpp csrc/keys/*.cpp csrc/zmq/*.cpp)
GPU_HOST   := $(wildcard csrc/gpu/*.cpp)
HIP_SRCS   := $(wildcard csrc/kernels/*.hip)
PY_SRCS    := $(wildcard csrc/python/*.cpp)
TOOL_SRCS  := $(wildcard csrc/tools/*.cpp)
TEST_SRCS  := $(wildcard csrc/test/*.cpp)

CORE_OBJS  := $(patsubst csrc/%.cpp,build/obj/%.o,$(CORE_SRCS) $(GPU_HOST))
HIP_OBJS   := $(patsubst csrc/%.hip,build/obj/%.o,$(HIP_SRCS))
PY_OBJS    := $(patsubst csrc/%.cpp,build/obj/%.o,$(PY_SRCS))
TOOLS      := $(patsubst csrc/tools/%.cpp,bin/%,$(TOOL_SRCS))
TEST_OBJS  := $(patsubst csrc/%.cpp,build/obj/%.o,$(TEST_SRCS))
UNITTEST   := bin/test_bcp

PYEXT      := bitcoincashplus_amd/_bcpnative$(PY_EXT)
CORELIB    := build/libbcpcore.a
CONSLIB    := lib/libbcpconsensus.so

.PHONY: all pyext tools clean kernels conslib unittest
.DEFAULT_GOAL := all
conslib: $(CONSLIB)
all: pyext tools conslib unittest
unittest: $(UNITTEST)
pyext: $(PYEXT)
kernels: $(HIP_OBJS)
tools: $(TOOLS)

build/obj/%.o: csrc/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -MMD -MP -c $< -o $@

build/obj/python/%.o: csrc/python/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -MMD -MP -c $< -o $@

build/obj/kernels/%.o: csrc/kernels/%.hip
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -MMD -MP -c $< -o $@

# Per-kernel-file flags. The Equihash solver: the max-ILP scheduler with the AMDGPU register
# pressure trackers, and no atomic optimizer (its loops around single-lane and per-thread
# atomics are pure overhead here): +1.8% Sol/s over the default codegen in interleaved A/Bs
# (profiles/equihash_r6.md).
HIPFLAGS_equihash_solver := -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers=1 \
                            -mllvm -amdgpu-atomic-optimizer-strategy=None

$(CORELIB): $(CORE_OBJS) $(HIP_OBJS)
	@mkdir -p $(dir $@)
	rm -f $@ && ar rcs $@ $^

$(PYEXT): $(PY_OBJS) $(CORELIB)
	$(CXX) -shared -o $@ $(PY_OBJS) -Wl,--whole-archive $(CORELIB) -Wl,--no-whole-archive $(LDLIBS) $(HARDEN_LD)

bin/%: build/obj/tools/%.o $(CORELIB)
	@mkdir -p bin
	$(CXX) -rdynamic -o $@ $< -Wl,--whole-archive $(CORELIB) -Wl,--no-whole-archive $(LDLIBS) $(HARDEN_LD)

# native unit suites (reference src/test/ -> test_bitcoin); run by tests/test_unit_native.py
$(UNITTEST): $(TEST_OBJS) $(CORELIB)
	@mkdir -p bin
	$(CXX) -rdynamic -o $@ $(TEST_OBJS) -Wl,--whole-archive $(CORELIB) -Wl,--no-whole-archive $(LDLIBS)

build/obj/tools/%.o: csrc/tools/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -MMD -MP -c $< -o $@

$(CONSLIB): build/obj/consensuslib/bitcoinconsensus.o $(CORELIB)
	@mkdir -p lib
	$(CXX) -shared -o $@ $< $(CORELIB) $(LDLIBS) $(HARDEN_LD)

# Host-side sanitizer build of the fuzz harness (reference --enable-asan/--enable-ubsan):
# every CPU source rebuilt with ASan+UBSan, the gfx950 kernel objects linked as they are
# (GPU code is never sanitized here).  `make asan` -> bin/bcp-fuzz-asan
ASAN_FLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -O1 -g
ASAN_OBJS  := $(patsubst csrc/%.cpp,build/asan/%.o,$(CORE_SRCS) $(GPU_HOST) csrc/tools/bcp-fuzz.cpp)
.PHONY: asan
asan: bin/bcp-fuzz-asan
build/asan/%.o: csrc/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(filter-out -O2,$(CXXFLAGS)) $(ASAN_FLAGS) -MMD -MP -c $< -o $@
bin/bcp-fuzz-asan: $(ASAN_OBJS) $(HIP_OBJS)
	@mkdir -p bin
	$(CXX) $(ASAN_FLAGS) -o $@ $^ $(LDLIBS)

# Host sanitizer builds of the node and the unit suites (reference --enable-tsan/--enable-asan,
# configure.ac:195-275): every CPU source rebuilt instrumented, the gfx950 kernel objects linked as
# they are.  `make tsan` -> bin/tsan/{bcpd,test_bcp}; `make asan-node` -> bin/asan/{bcpd,test_bcp}.
# tools/sanitize.sh runs the unit suites and the P2P/ConnectBlock functional tests under both.
TSAN_FLAGS := -fsanitize=thread -fno-omit-frame-pointer -O1 -g -include csrc/util/tsan_compat.h
SAN_SRCS   := $(CORE_SRCS) $(GPU_HOST)
TSAN_CORE  := $(patsubst csrc/%.cpp,build/tsan/%.o,$(SAN_SRCS))
TSAN_TEST  := $(patsubst csrc/%.cpp,build/tsan/%.o,$(TEST_SRCS))
ASAN_CORE  := $(patsubst csrc/%.cpp,build/asan/%.o,$(SAN_SRCS))
ASAN_TEST  := $(patsubst csrc/%.cpp,build/asan/%.o,$(TEST_SRCS))
.PHONY: tsan asan-node
tsan: bin/tsan/bcpd bin/tsan/test_bcp
asan-node: bin/asan/bcpd bin/asan/test_bcp
build/tsan/%.o: csrc/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(filter-out -O2,$(CXXFLAGS)) $(TSAN_FLAGS) -MMD -MP -c $< -o $@
bin/tsan/bcpd: build/tsan/tools/bcpd.o $(TSAN_CORE) $(HIP_OBJS)
	@mkdir -p bin/tsan
	$(CXX) $(TSAN_FLAGS) -rdynamic -o $@ $^ $(LDLIBS)
bin/tsan/test_bcp: $(TSAN_TEST) $(TSAN_CORE) $(HIP_OBJS)
	@mkdir -p bin/tsan
	$(CXX) $(TSAN_FLAGS) -rdynamic -o $@ $^ $(LDLIBS)
bin/asan/bcpd: build/asan/tools/bcpd.o $(ASAN_CORE) $(HIP_OBJS)
	@mkdir -p bin/asan
	$(CXX) $(ASAN_FLAGS) -rdynamic -o $@ $^ $(LDLIBS)
bin/asan/test_bcp: $(ASAN_TEST) $(ASAN_CORE) $(HIP_OBJS)
	@mkdir -p bin/asan
	$(CXX) $(ASAN_FLAGS) -rdynamic -o $@ $^ $(LDLIBS)

# Clang thread-safety analysis over every CPU source (reference src/threadsafety.h, built with
# -Wthread-safety under clang): GUARDED_BY / EXCLUSIVE_LOCKS_REQUIRED / LOCKS_EXCLUDED on the
# chainstate, mempool and connection manager; any warning fails the target.
TSA_CXX    ?= $(ROCM)/lib/llvm/bin/clang++
TSA_STAMPS := $(patsubst csrc/%.cpp,build/tsa/%.ok,$(SAN_SRCS))
.PHONY: thread-safety
thread-safety: $(TSA_STAMPS)
build/tsa/%.ok: csrc/%.cpp
	@mkdir -p $(dir $@)
	$(TSA_CXX) -std=c++17 -fsyntax-only -Icsrc -Wthread-safety -Werror=thread-safety -Wno-unknown-warning-option \
	    -MMD -MP -MF $(@:.ok=.d) -MT $@ $<
	@touch $@

clean:
	rm -rf build bin lib bitcoincashplus_amd/_bcpnative*.so

-include $(shell find build -name '*.d' 2>/dev/null)
