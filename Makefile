# Host-side sanitizer build (SURVEY.md §5 "Race detection / sanitizers"):
#   make asan
# builds into build/asan/ (not shipped to GPU runs), with AddressSanitizer +
# UndefinedBehaviorSanitizer,
#   build/asan/libdtsim_asan.so    libdtsim with its HOST code instrumented
#                                 (argument checks, map validation, handle
#                                 bookkeeping); the gfx950 device code is
#                                 compiled as usual, uninstrumented
#                                 (-fno-gpu-sanitize)
#   build/asan/liboracle_asan.so  the oracle's C restatement (test
#                                 infrastructure), with the same runtime
# Both use clang's ASan runtime (which carries UBSan's), preloaded into the
# process that loads them (tests/test_asan.py: LD_PRELOAD=$(ASAN_RT)).
# GPU sanitizers (GPU ASan, xnack+) are not available on the GPU pool.
HIPCC ?= /opt/rocm/bin/hipcc
CLANG ?= /opt/rocm/lib/llvm/bin/clang
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
HIP_SAN := --offload-arch=gfx950 -O1 -fsanitize=address,undefined -fno-gpu-sanitize \
  -fno-sanitize-recover=undefined -Xarch_host -g -Xarch_host -fno-omit-frame-pointer
SRCS := $(wildcard aido1_amd/csrc/*.hip)
HDRS := $(wildcard aido1_amd/csrc/*.h) $(wildcard include/*.h)
OBJS := $(patsubst aido1_amd/csrc/%.hip,build/asan/%.o,$(SRCS))
ORACLE_SRCS := $(wildcard oracle/*.c)

.PHONY: asan asan-rt clean-asan
asan: build/asan/libdtsim_asan.so build/asan/liboracle_asan.so

asan-rt:
	@$(CLANG) -print-file-name=libclang_rt.asan-x86_64.so

build/asan/%.o: aido1_amd/csrc/%.hip $(HDRS)
	@mkdir -p build/asan
	$(HIPCC) $(HIP_SAN) -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -c $< -o $@

build/asan/libdtsim_asan.so: $(OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(OBJS)

build/asan/liboracle_asan.so: $(ORACLE_SRCS) include/dtsim.h
	@mkdir -p build/asan
	$(CLANG) -shared -fPIC -std=c11 -ffp-contract=off -fno-fast-math -fno-builtin -Wall $(SAN) \
	  -o $@ $(ORACLE_SRCS) -lm

clean-asan:
	rm -rf build/asan
