# MI355X (gfx950) cipher engine -- native build.
#
#   make            -> our_tree_amd/lib/libotc.so (HIP kernels + runtime + CPU oracle)
#                      our_tree_amd/lib/libotc_cpu.so (CPU oracle only, no ROCm deps)
#                      bin/test bin/aes_test bin/aes_ecb_e bin/aes_ecb_d bin/otbench bin/bc_test
#   make cpu        -> CPU-only pieces (no hipcc needed)
#   make SAN=1 cpu  -> CPU oracle with ASan/UBSan (host only)
#   make SAN=thread cpu -> CPU oracle with ThreadSanitizer (host only)
#   make san-check  -> build csrc/cli/san_driver.c with TSan and ASan+UBSan, run both
#
# Reference build: Makefile:1-56 (gcc -O0), aes-modes/Makefile (clang -O0,
# broken on current compilers), aes-gpu/Source/Makefile.asc (nvcc, no -arch).
ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
CXX     ?= g++

INC      := -Icsrc/include -Icsrc/hip
CFLAGS   ?= -O2 -g -Wall -Wextra -std=gnu99 -fPIC
CXXFLAGS ?= -O2 -g -Wall -std=c++17 -fPIC
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SANLD :=
ifeq ($(SAN),1)
CFLAGS   += -fsanitize=address,undefined -fno-omit-frame-pointer
CXXFLAGS += -fsanitize=address,undefined -fno-omit-frame-pointer
SANLD    := -fsanitize=address,undefined
endif
ifeq ($(SAN),thread)
CFLAGS   += -fsanitize=thread
CXXFLAGS += -fsanitize=thread
SANLD    := -fsanitize=thread
endif

LIBDIR := our_tree_amd/lib
OBJ    := build/obj

CPU_SRC := csrc/cpu/aes.c csrc/cpu/arc4.c csrc/cpu/rc4.c csrc/cpu/aesni.c csrc/cpu/numa.c csrc/cpu/rccl_plan.c
CPU_OBJ := $(patsubst csrc/cpu/%.c,$(OBJ)/cpu/%.o,$(CPU_SRC)) $(OBJ)/cpu/bs_selftest.o
HIP_SRC := csrc/hip/aes_tt.hip csrc/hip/aes_bs.hip csrc/hip/stream_ops.hip
HIP_OBJ := $(patsubst csrc/hip/%.hip,$(OBJ)/hip/%.o,$(HIP_SRC)) $(OBJ)/hip/engine.o $(OBJ)/hip/pipeline.o

BINS := bin/test bin/aes_test bin/aes_ecb_e bin/aes_ecb_d bin/otbench bin/bc_test

.PHONY: all cpu clean
all: $(LIBDIR)/libotc.so $(LIBDIR)/libotc_cpu.so $(BINS) bin/test_cpu bin/aes_test_cpu bin/otbench_hostsim ref-o0
cpu: $(LIBDIR)/libotc_cpu.so bin/test_cpu bin/aes_test_cpu bin/otbench_hostsim ref-o0

$(OBJ)/cpu/aesni.o: csrc/cpu/aesni.c csrc/include/aesni.h
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -maes -msse4.1 -mssse3 $(INC) -c $< -o $@

$(OBJ)/cpu/%.o: csrc/cpu/%.c $(wildcard csrc/include/*.h)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) $(INC) -c $< -o $@

$(OBJ)/cpu/bs_selftest.o: csrc/cpu/bs_selftest.cpp $(wildcard csrc/include/*.h)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -Wno-unknown-pragmas $(INC) -c $< -o $@

# -fno-slp-vectorize: the SLP vectorizer packs the 4 independent transposes /
# 16 S-boxes of the bitsliced kernel into lock-stepped vector ops, which doubles
# the live register set (1 wave/SIMD + AGPR spills).  See docs/PERF.md.
$(OBJ)/hip/aes_bs.o: HIPFLAGS += -fno-slp-vectorize

$(OBJ)/hip/%.o: csrc/hip/%.hip $(wildcard csrc/hip/*.h) $(wildcard csrc/include/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(INC) -c $< -o $@

$(OBJ)/hip/%.o: csrc/hip/%.cpp csrc/hip/otc_device.h csrc/hip/engine_internal.h $(wildcard csrc/include/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip $(INC) -c $< -o $@

$(LIBDIR)/libotc.so: $(HIP_OBJ) $(CPU_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -L$(ROCM)/lib -lrccl -lrocprofiler-sdk-roctx -lpthread -Wl,--no-undefined -Wl,-rpath,$(ROCM)/lib

$(LIBDIR)/libotc_cpu.so: $(CPU_OBJ)
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -fPIC -o $@ $^ -lpthread $(SANLD)

# --- CLIs -------------------------------------------------------------------
bin/test_cpu: csrc/cli/rc4_test.c $(CPU_OBJ)
	@mkdir -p bin
	$(CXX) -O2 $(INC) -x c -std=gnu99 $< -x none $(CPU_OBJ) -o $@ -lpthread $(SANLD)

bin/aes_test_cpu: csrc/cli/aes_test.c $(CPU_OBJ)
	@mkdir -p bin
	$(CXX) -O2 $(INC) -x c -std=gnu99 $< -x none $(CPU_OBJ) -o $@ -lpthread $(SANLD)

bin/test: csrc/cli/rc4_test.c $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CC) -O2 -std=gnu99 -DOTC_WITH_GPU $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

bin/aes_test: csrc/cli/aes_test.c $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CC) -O2 -std=gnu99 -DOTC_WITH_GPU $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

bin/aes_ecb_e: csrc/cli/aes_ecb_e.c $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CC) -O2 -std=gnu99 $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

bin/aes_ecb_d: csrc/cli/aes_ecb_d.c $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CC) -O2 -std=gnu99 $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

bin/otbench: csrc/cli/otbench.cpp $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

# otbench over a host-memory double of the device API (CPU tests of its
# argument / snapshot / verification logic, tests/test_otbench_cpu.py)
bin/otbench_hostsim: csrc/cli/otbench.cpp csrc/cli/otc_hostsim.cpp $(CPU_OBJ)
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 -Wall $(INC) csrc/cli/otbench.cpp csrc/cli/otc_hostsim.cpp $(CPU_OBJ) -o $@ -lpthread

bin/bc_test: csrc/cli/bc_test.cpp csrc/include/otc_cipher.hpp $(LIBDIR)/libotc.so
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 -Wall $(INC) $< -o $@ -L$(LIBDIR) -lotc -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# --- reference-methodology CPU baseline --------------------------------------
# The reference's published CPU numbers were built at -O0 (reference
# Makefile:13 "gcc -g -Wall -pedantic -O0 -std=gnu99", aes-modes/Makefile:15
# "clang -O0 -msse4.1 -maes").  bin/test_o0 and bin/aes_test_o0 are the same
# harnesses and oracle built the same way, for apples-to-apples rows against
# the results.* logs (the -O2 builds above are the real CPU baseline).
O0FLAGS := -g -Wall -pedantic -O0 -std=gnu99
O0_OBJ  := $(patsubst csrc/cpu/%.c,$(OBJ)/o0/%.o,$(CPU_SRC)) $(OBJ)/o0/bs_selftest.o
# --- A/B variant libraries ------------------------------------------------
# make variant NAME=b4 VFLAGS="-DOTC_TT_CLAIM_B=4"  ->  variants/b4/libotc.so
# (its own object dir; load it with OTC_LIB=variants/b4/libotc.so).  A/B
# switches are compile-time: the production library carries no env knobs.
.PHONY: variant
variant:
	@test -n "$(NAME)" || (echo "NAME=... required" && false)
	$(MAKE) OBJ=build/obj-$(NAME) LIBDIR=variants/$(NAME) HIPFLAGS="$(HIPFLAGS) $(VFLAGS)" variants/$(NAME)/libotc.so

.PHONY: ref-o0
ref-o0: bin/test_o0 bin/aes_test_o0

$(OBJ)/o0/aesni.o: csrc/cpu/aesni.c csrc/include/aesni.h
	@mkdir -p $(dir $@)
	$(CC) $(O0FLAGS) -maes -msse4.1 -mssse3 $(INC) -c $< -o $@

$(OBJ)/o0/%.o: csrc/cpu/%.c $(wildcard csrc/include/*.h)
	@mkdir -p $(dir $@)
	$(CC) $(O0FLAGS) $(INC) -c $< -o $@

$(OBJ)/o0/bs_selftest.o: csrc/cpu/bs_selftest.cpp csrc/include/otc_bitslice.h
	@mkdir -p $(dir $@)
	$(CXX) -g -O0 -std=c++17 $(INC) -c $< -o $@

bin/test_o0: csrc/cli/rc4_test.c $(O0_OBJ)
	@mkdir -p bin
	$(CXX) -O0 -g $(INC) -x c -std=gnu99 $< -x none $(O0_OBJ) -o $@ -lpthread

bin/aes_test_o0: csrc/cli/aes_test.c $(O0_OBJ)
	@mkdir -p bin
	$(CXX) -O0 -g $(INC) -x c -std=gnu99 $< -x none $(O0_OBJ) -o $@ -lpthread

clean:
	rm -rf build $(LIBDIR)/*.so $(BINS) bin/otbench_hostsim bin/test_cpu bin/aes_test_cpu bin/test_o0 bin/aes_test_o0

# Host sanitizers over the threaded CPU paths (also tests/test_sanitizers_cpu.py)
SAN_SRC := csrc/cpu/aes.c csrc/cpu/arc4.c csrc/cli/san_driver.c
san-check:
	@mkdir -p build/san
	$(CC) -O1 -g -std=gnu99 -Icsrc/include -fsanitize=thread $(SAN_SRC) -o build/san/tsan -lpthread
	$(CC) -O1 -g -std=gnu99 -Icsrc/include -fsanitize=address,undefined -fno-sanitize-recover=undefined $(SAN_SRC) -o build/san/asan -lpthread
	TSAN_OPTIONS=halt_on_error=1 ./build/san/tsan
	./build/san/asan
.PHONY: san-check
