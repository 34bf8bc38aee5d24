# Host-side sanitizer builds: AddressSanitizer + UBSan on the
# oracle (oracle/dronerl_oracle.c) and on libdronerl's host code (the C ABI's
# argument validation, layout queries, handle lifecycle), then the CPU test
# suite with both loaded.  GPU code is not instrumented (-Xarch_host): GPU
# sanitizers are not available on the MI355X pool.  One ASan runtime (clang's)
# is preloaded into python for both libraries.
#
#   make asan        build build/asan/liboracle.so and build/asan/libdronerl.so
#   make asan-test   run `pytest -m "not gpu"` against them
ROCM ?= /opt/rocm
CLANG := $(ROCM)/llvm/bin/clang
HIPCC := $(ROCM)/bin/hipcc
ASAN_RT := $(shell $(CLANG) -print-file-name=libclang_rt.asan-x86_64.so)
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer
HOSTSAN := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
           -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer
CSRC := dronerl_amd/csrc
SRCS := $(CSRC)/dronerl_kernels.hip $(CSRC)/dronerl_api.cpp $(CSRC)/dronerl_env.cpp $(CSRC)/dronerl_qnet.hip \
        $(CSRC)/dronerl_qnet_api.cpp $(CSRC)/dronerl_learn.hip
DEPS := $(SRCS) $(CSRC)/dronerl_internal.h include/dronerl.h

asan: build/asan/liboracle.so build/asan/libdronerl.so

build/asan/liboracle.so: oracle/dronerl_oracle.c
	@mkdir -p build/asan
	$(CLANG) -O1 -g -std=c11 -fPIC -shared -shared-libsan $(SAN) -o $@ $< -lm -lpthread

build/asan/libdronerl.so: $(DEPS)
	@mkdir -p build/asan
	$(HIPCC) --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -shared-libsan $(HOSTSAN) -I include -o $@ $(SRCS)

asan-test: asan
	ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	LD_PRELOAD=$(ASAN_RT) DRL_LIB=$(CURDIR)/build/asan/libdronerl.so DRL_ORACLE_LIB=$(CURDIR)/build/asan/liboracle.so \
	python -m pytest tests -m "not gpu" -q -p no:cacheprovider

.PHONY: asan asan-test
