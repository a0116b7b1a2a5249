# Native build of veles.simd_amd: one shared library (C API + HIP kernels for
# gfx950) and the native C API test binary.  Driven by
# `python -m veles.simd_amd.build` / __graft_entry__.build(); plain `make -j`
# works too.
#
# Copyright 2026 veles.simd_amd authors. Apache-2.0.

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
BUILD    ?= build
LIBDIR   := veles/simd_amd/_native
LIB      := $(LIBDIR)/libvelessimd.so
OPT      ?= -O3
LDEXTRA  ?=

COMMON   := $(OPT) -std=c++17 -fPIC -I. -Iinclude -Wall -Wextra \
            -Wno-unused-parameter -Wno-unused-command-line-argument \
            -DVELES_SIMD_IMPLEMENTATION -fvisibility=hidden
# -packed-fp32-ops: the compiler emits no v_pk_{add,mul,fma}_f32 (some forms
# of these have returned wrong results on this hardware pool).
HIPFLAGS := $(COMMON) -x hip --offload-arch=$(ARCH) \
            -ffp-contract=fast -Xclang -target-feature -Xclang -packed-fp32-ops
CXXFLAGS := $(COMMON) -ffp-contract=off

HIP_SRCS := $(sort $(wildcard csrc/kernels/*.hip))
CPP_SRCS := $(sort $(wildcard csrc/runtime/*.cpp csrc/ref/*.cpp \
              csrc/api/*.cpp csrc/data/*.cpp csrc/dist/*.cpp))
HIP_OBJS := $(patsubst %.hip,$(BUILD)/%.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst %.cpp,$(BUILD)/%.o,$(CPP_SRCS))
HEADERS  := $(wildcard include/simd/*.h csrc/*/*.h)

TEST_BIN := $(BUILD)/tests/capi_test

.PHONY: all lib tests clean

all: lib tests

lib: $(LIB)

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -Wl,-soname,libvelessimd.so \
	    -L/opt/rocm/lib -lrccl -lmvec -lm -Wl,-rpath,/opt/rocm/lib $(LDEXTRA)

$(BUILD)/%.o: %.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: %.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

tests: $(TEST_BIN)

$(TEST_BIN): tests/native/capi_test.cpp $(LIB) $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) -O2 -std=c++17 -Iinclude -Itests/native $< -o $@ \
	    -L$(LIBDIR) -lvelessimd -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'
	$(HIPCC) -O2 -std=c++17 -Iinclude -Itests/native tests/native/threads_test.cpp \
	    -o $(dir $@)threads_test -L$(LIBDIR) -lvelessimd -lpthread \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

clean:
	rm -rf $(BUILD) $(LIB)

# Install: library + the public headers + pkg-config file, the layout of
# the reference's `make install` (/root/reference/inc/Makefile.am:27-31,
# src/Makefile.am:29, Simd.pc.in).  The library is also installed as
# libSimd.so and the .pc as Simd.pc, so `pkg-config --cflags --libs Simd`
# and `-lSimd` consumers of the reference link unchanged.
#   make install PREFIX=/opt/veles [DESTDIR=/tmp/stage]
PREFIX     ?= /usr/local
DESTDIR    ?=
VERSION    := $(shell sed -n 's/^__version__ = "\(.*\)"/\1/p' veles/simd_amd/__init__.py)
INST_LIB   := $(DESTDIR)$(PREFIX)/lib
INST_INC   := $(DESTDIR)$(PREFIX)/include/simd
INST_PC    := $(INST_LIB)/pkgconfig
install: $(LIB)
	install -d $(INST_LIB) $(INST_INC) $(INST_PC)
	install -m 0755 $(LIB) $(INST_LIB)/libvelessimd.so.$(VERSION)
	ln -sf libvelessimd.so.$(VERSION) $(INST_LIB)/libvelessimd.so
	ln -sf libvelessimd.so.$(VERSION) $(INST_LIB)/libSimd.so
	install -m 0644 include/simd/*.h $(INST_INC)/
	sed -e 's|@prefix@|$(PREFIX)|' -e 's|@libdir@|$(PREFIX)/lib|' \
	    -e 's|@includedir@|$(PREFIX)/include|' -e 's|@VERSION@|$(VERSION)|' \
	    -e 's|@rocmlib@|/opt/rocm/lib|' simd.pc.in > $(INST_PC)/Simd.pc
	ln -sf Simd.pc $(INST_PC)/veles-simd-amd.pc

uninstall:
	rm -f $(INST_LIB)/libvelessimd.so* $(INST_LIB)/libSimd.so $(INST_PC)/Simd.pc \
	    $(INST_PC)/veles-simd-amd.pc
	rm -rf $(INST_INC)

# Static analysis (clang analyzer + strict warnings, host side of every
# source); report in build/lint/report.txt.
lint:
	bash tools/lint.sh

# API reference (Doxygen, if installed) into build/docs.
docs:
	@command -v doxygen >/dev/null || { echo "doxygen not installed"; exit 1; }
	mkdir -p $(BUILD)/docs && doxygen docs/Doxyfile

.PHONY: install uninstall lint docs

# Host AddressSanitizer build of the library + native C API test (host code
# only: device ASan / XNACK is not available on the GPU pool).  Runs the
# host-reference paths on any machine: `make asan && ASAN_OPTIONS=detect_leaks=1 \
#   VELES_DISABLE_GPU=1 build-asan/tests/capi_test`.
ASAN_BUILD := build-asan
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer
asan:
	$(MAKE) BUILD=$(ASAN_BUILD) OPT="$(ASAN_FLAGS) -Xarch_host -fsanitize=address" \
	    LIBDIR=$(ASAN_BUILD)/lib LIB=$(ASAN_BUILD)/lib/libvelessimd.so \
	    TEST_BIN=$(ASAN_BUILD)/tests/capi_test lib
	@mkdir -p $(ASAN_BUILD)/tests
	$(HIPCC) $(ASAN_FLAGS) -Xarch_host -fsanitize=address -std=c++17 -Iinclude -Itests/native \
	    tests/native/capi_test.cpp -o $(ASAN_BUILD)/tests/capi_test \
	    -L$(ASAN_BUILD)/lib -lvelessimd -Wl,-rpath,'$$ORIGIN/../lib'

.PHONY: asan

# Host ThreadSanitizer build + the multi-threaded native test (host code only).
#   make tsan && VELES_DISABLE_GPU=1 build-tsan/tests/threads_test 8 5
TSAN_BUILD := build-tsan
TSAN_FLAGS := -O1 -g -fno-omit-frame-pointer
tsan:
	$(MAKE) BUILD=$(TSAN_BUILD) OPT="$(TSAN_FLAGS) -Xarch_host -fsanitize=thread" \
	    LIBDIR=$(TSAN_BUILD)/lib LIB=$(TSAN_BUILD)/lib/libvelessimd.so \
	    LDEXTRA=-fsanitize=thread TEST_BIN=$(TSAN_BUILD)/tests/capi_test lib
	@mkdir -p $(TSAN_BUILD)/tests
	$(HIPCC) $(TSAN_FLAGS) -Xarch_host -fsanitize=thread -std=c++17 -Iinclude -Itests/native \
	    tests/native/threads_test.cpp -o $(TSAN_BUILD)/tests/threads_test \
	    -L$(TSAN_BUILD)/lib -lvelessimd -lpthread -Wl,-rpath,'$$ORIGIN/../lib'

.PHONY: tsan

# Host UndefinedBehaviorSanitizer build (shared runtime, so the CPU pytest suite can load
# the library into an uninstrumented python; any finding aborts):
#   make ubsan && VELES_SIMD_LIB=$PWD/build-ubsan/lib/libvelessimd.so VELES_DISABLE_GPU=1 \
#     python -m pytest tests -m "not gpu" -p no:cacheprovider
UBSAN_BUILD := build-ubsan
UBSAN_RT    := $(dir $(shell /opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.ubsan_standalone-x86_64.so))
ubsan:
	$(MAKE) BUILD=$(UBSAN_BUILD) LIBDIR=$(UBSAN_BUILD)/lib LIB=$(UBSAN_BUILD)/lib/libvelessimd.so \
	    OPT="-O1 -g -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined" \
	    LDEXTRA="-fsanitize=undefined -shared-libsan -Wl,-rpath,$(UBSAN_RT)" lib

.PHONY: ubsan

# Host line coverage (gcov), the counterpart of the reference's
# --enable-test-coverage (common.ac:229-236): host code of every source built
# with --coverage, then the native C test and the CPU pytest suite run
# against that library; per-file line coverage in build-cov/coverage.txt.
#   make coverage            (no GPU needed: host-reference paths)
COV_BUILD := build-cov
COV_FLAGS := -O2 -g -Xarch_host --coverage
coverage:
	$(MAKE) BUILD=$(COV_BUILD) OPT="$(COV_FLAGS)" LDEXTRA=--coverage \
	    LIBDIR=$(COV_BUILD)/lib LIB=$(COV_BUILD)/lib/libvelessimd.so lib
	@mkdir -p $(COV_BUILD)/tests
	$(HIPCC) -O2 -g -std=c++17 -Iinclude -Itests/native \
	    tests/native/capi_test.cpp -o $(COV_BUILD)/tests/capi_test \
	    -L$(COV_BUILD)/lib -lvelessimd -Wl,-rpath,'$$ORIGIN/../lib'
	find $(COV_BUILD) -name '*.gcda' -delete
	VELES_DISABLE_GPU=1 $(COV_BUILD)/tests/capi_test > $(COV_BUILD)/capi_test.log
	VELES_SIMD_LIB=$(CURDIR)/$(COV_BUILD)/lib/libvelessimd.so VELES_DISABLE_GPU=1 \
	    python -m pytest tests -m "not gpu" -q -p no:cacheprovider > $(COV_BUILD)/pytest.log
	python tools/coverage_report.py $(COV_BUILD) > $(COV_BUILD)/coverage.txt
	tail -n 30 $(COV_BUILD)/coverage.txt

.PHONY: coverage

# Diagnostic build: per-phase s_memtime stamps in the real-block conv kernel
# (tools/conv_stamps.py).  Not the shipped library.
STAMPS_BUILD := build-stamps
stamps:
	$(MAKE) BUILD=$(STAMPS_BUILD) OPT="-O3 -DVS_CONV_STAMPS" \
	    LIBDIR=$(STAMPS_BUILD)/lib LIB=$(STAMPS_BUILD)/lib/libvelessimd.so lib

.PHONY: stamps

# Diagnostic build: timing-only SGEMM ablations (compile-time bits ABLATE=4|8|16 drop
# the in-loop barriers / DMA pieces / fragment reads of the gen-7 kernel;
# results are wrong by design).  Not the shipped library.
ABLATE      ?= 4
ABLATE_BUILD := build-ablate/$(ABLATE)
ablate:
	$(MAKE) BUILD=$(ABLATE_BUILD) OPT="-O3 -DVS_SGEMM_ABLATE=$(ABLATE)" \
	    LIBDIR=$(ABLATE_BUILD)/lib LIB=$(ABLATE_BUILD)/lib/libvelessimd.so lib

.PHONY: ablate
