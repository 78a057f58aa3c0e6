# Builds the MI355X (gfx950) sampling path: librtw.so (C ABI, include/rtw_capi.h),
# the rtw_cli driver (mirrors the reference's main.rs), and the test-only oracle.
# Everything f64 is compiled with -ffp-contract=off (no FMA contraction): parity
# with the reference's generic x86-64 release build depends on it.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
# xnack- : the pool runs without XNACK (no page-fault retry), and code built for it is
# free of the xnack-any constraints: 127.9 -> 127.5 ms per image, 8-round A/B
# (profiles/r02_misc/ab_xnack_off.log). Such a code object does not load on a gfx950
# running with XNACK enabled: `make ARCH=gfx950` builds the portable (xnack-any) one.
# (A fat binary with an xnack+ object beside it is not an option here: the GPU pool
# refuses any tree that carries xnack+ code.) ARCH may list several targets;
# rtw_version() names the target features the library carries.
ARCH ?= gfx950:xnack-
PKG := raytracing_in_a_weekend_rust_amd
SRC := $(PKG)/csrc
OUT := $(PKG)/_lib
ARCHFLAGS := $(foreach a,$(ARCH),--offload-arch=$(a))
HIPFLAGS_1 := -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
            -Wall -Iinclude -I$(SRC) -I$(SRC)/host $(EXTRA)
HIPFLAGS := $(ARCHFLAGS) $(HIPFLAGS_1)
CXXFLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wextra \
            -Iinclude -I$(SRC)/host -D__HIP_PLATFORM_AMD__
# Build id: hash of every library source and the device flags. rtw_build_id()
# returns it; profiles/ PMC files are stamped with it and bench.py refuses a file
# whose stamp differs from the loaded library's.
LIB_SRCS := $(sort $(wildcard $(SRC)/*.hip $(SRC)/*.h $(SRC)/host/*.cpp $(SRC)/host/*.h)) include/rtw_capi.h
BUILD_ID := $(shell cat $(LIB_SRCS) | sha256sum | cut -c1-12)-$(shell echo '$(ARCH) $(HIPFLAGS)' | sha256sum | cut -c1-4)

all: $(OUT)/librtw.so $(OUT)/rtw_cli oracle $(OUT)/accel_check $(OUT)/next01_check $(OUT)/try_check $(OUT)/karg_check.ok

$(OUT)/rtw_render.o: $(SRC)/rtw_render.hip $(SRC)/rtw_fast.h $(SRC)/rtw_accel.h $(SRC)/rtw_numeric.h include/rtw_capi.h $(SRC)/host/rtw_host.h $(SRC)/host/rtw_internal.h
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# f32 fast mode: FMA contraction allowed (its own file, its own flags)
$(OUT)/rtw_fast.o: $(SRC)/rtw_fast.hip $(SRC)/rtw_fast.h $(SRC)/rtw_accel.h include/rtw_capi.h
	@mkdir -p $(OUT)
	$(HIPCC) $(filter-out -ffp-contract=off,$(HIPFLAGS)) -ffp-contract=fast -c $< -o $@

# multi-GPU groups (RCCL gather, opened with dlopen at first use)
$(OUT)/rtw_group.o: $(SRC)/rtw_group.hip include/rtw_capi.h $(SRC)/host/rtw_internal.h
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/rtw_accel_build.o: $(SRC)/host/rtw_accel_build.cpp $(SRC)/rtw_accel.h
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -I$(SRC) -c $< -o $@

# test infrastructure: exhaustive check of the division-free next_01 (tests/test_accel.py)
$(OUT)/next01_check: tools/next01_check.cpp $(SRC)/rtw_numeric.h
	@mkdir -p $(OUT)
	$(CXX) -O2 -std=c++17 -ffp-contract=off -fno-fast-math -I$(SRC) -o $@ $< -lpthread

# test infrastructure: host emulation of the trapped-path replay vs the serial draws (tests/test_accel.py)
$(OUT)/try_check: tools/try_check.cpp $(SRC)/rtw_numeric.h $(OUT)/librtw.so
	$(CXX) $(CXXFLAGS) -I$(SRC) -o $@ tools/try_check.cpp -L$(OUT) -lrtw -Wl,-rpath,'$$ORIGIN'

# test infrastructure: host self-check of the BVH walk (tests/test_accel.py)
$(OUT)/accel_check: tools/accel_check.cpp $(OUT)/rtw_accel_build.o $(OUT)/librtw.so
	$(CXX) $(CXXFLAGS) -I$(SRC) -o $@ tools/accel_check.cpp $(OUT)/rtw_accel_build.o -L$(OUT) -lrtw -Wl,-rpath,'$$ORIGIN'

# rewritten only when the id changes (so an unchanged tree rebuilds nothing)
$(OUT)/rtw_build_id.h: FORCE
	@mkdir -p $(OUT)
	@echo '#define RTW_BUILD_ID "$(BUILD_ID)"' > $@.tmp
	@echo '#define RTW_BUILD_ARCH "$(ARCH)"' >> $@.tmp
	@cmp -s $@.tmp $@ || mv $@.tmp $@
	@rm -f $@.tmp

$(OUT)/rtw_host.o: $(SRC)/host/rtw_host.cpp include/rtw_capi.h $(SRC)/host/rtw_host.h $(SRC)/host/rtw_internal.h $(OUT)/rtw_build_id.h
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -I$(OUT) -c $< -o $@

$(OUT)/librtw.so: $(OUT)/rtw_render.o $(OUT)/rtw_fast.o $(OUT)/rtw_group.o $(OUT)/rtw_host.o $(OUT)/rtw_accel_build.o
	$(HIPCC) $(ARCHFLAGS) -shared -fPIC -o $@ $^ -Wl,-soname,librtw.so -lpthread -ldl

$(OUT)/rtw_cli: $(SRC)/host/rtw_cli.cpp $(OUT)/librtw.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lrtw -Wl,-rpath,'$$ORIGIN' -lpthread

oracle:
	$(MAKE) -C oracle

# diagnostic build with per-wave s_memtime section stamps (tools/stamps.py)
stamps: $(OUT)/librtw_stamps.so
$(OUT)/rtw_render_stamps.o: $(SRC)/rtw_render.hip include/rtw_capi.h $(SRC)/host/rtw_host.h
	$(HIPCC) $(HIPFLAGS) -DRTW_STAMPS -c $< -o $@
# its own host object: rtw_build_id() carries "+stamps" (the diagnostic
# library must not report the default build's id)
$(OUT)/rtw_host_stamps.o: $(SRC)/host/rtw_host.cpp include/rtw_capi.h $(SRC)/host/rtw_host.h $(SRC)/host/rtw_internal.h $(OUT)/rtw_build_id.h
	$(CXX) $(CXXFLAGS) -I$(OUT) '-DRTW_BUILD_VARIANT="+stamps"' -c $< -o $@
$(OUT)/librtw_stamps.so: $(OUT)/rtw_render_stamps.o $(OUT)/rtw_fast.o $(OUT)/rtw_group.o $(OUT)/rtw_host_stamps.o $(OUT)/rtw_accel_build.o
	$(HIPCC) $(ARCHFLAGS) -shared -fPIC -o $@ $^ -Wl,-soname,librtw_stamps.so -lpthread

RENDER_DEPS := $(SRC)/rtw_render.hip $(SRC)/rtw_fast.h $(SRC)/rtw_accel.h $(SRC)/rtw_numeric.h include/rtw_capi.h $(SRC)/host/rtw_host.h $(SRC)/host/rtw_internal.h
asm: build/rtw_render.s
build/rtw_render.s: $(RENDER_DEPS)
	@mkdir -p build
	$(HIPCC) --offload-arch=$(firstword $(ARCH)) $(HIPFLAGS_1) --cuda-device-only -S -o $@ $<

# Build-time guard of KP()/CamRef: every function of the render
# file that reads KParams through the kernarg segment must be a lone-KParams kernel
# without calls (tools/check_karg.py). Part of `all`: an outlined helper fails the build.
$(OUT)/karg_check.ok: build/rtw_render.s tools/check_karg.py
	@mkdir -p $(OUT)
	python3 tools/check_karg.py build/rtw_render.s
	@touch $@
# its self-test: write_pixel deliberately noinline (RTW_KARG_SELFTEST) must be rejected
karg-selftest: $(RENDER_DEPS) tools/check_karg.py
	@mkdir -p build
	$(HIPCC) --offload-arch=$(firstword $(ARCH)) $(HIPFLAGS_1) -DRTW_KARG_SELFTEST --cuda-device-only -S -o build/rtw_render_selftest.s $<
	python3 tools/check_karg.py build/rtw_render_selftest.s --expect-fail

# A/B variant of the library (tools/libab.py): make ablib NAME=x EXTRA=-DFOO -> ab/x/librtw.so
ablib:
	$(MAKE) OUT=ab/$(NAME) EXTRA='$(EXTRA)' ab/$(NAME)/librtw.so

clean:
	rm -rf $(OUT) build
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean stamps ablib karg-selftest FORCE
FORCE:
