# liborbgpu.so: the MI355X (gfx950) ORB front-end.  `make` here or __graft_entry__.build().
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := orbslam3lib_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
# MFMA accumulators in VGPRs (k_knn2_mfma reads every result: no v_accvgpr copies)
DEVFLAGS := -mllvm -amdgpu-mfma-vgpr-form
LIB := orbslam3lib_amd/liborbgpu.so
HDRS := $(wildcard $(CSRC)/*.h) include/orbgpu.h

all: $(LIB) oracle facade_test idl_test

# one object per translation unit (each launcher sits beside its kernels: no relocatable device
# code needed), so `make -j` compiles them in parallel
LIBSRC := orb_kernels.hip orb_stereo.hip orb_frame.hip orb_io.hip orb_sbp.hip orb_fisheye.hip orb_runtime.cpp
OBJDIR := $(CSRC)/build
LIBOBJ := $(patsubst %,$(OBJDIR)/%.o,$(LIBSRC))

$(OBJDIR)/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -c -o $@ $<

$(LIB): $(LIBOBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(LIBOBJ)

oracle:
	$(MAKE) -s -C oracle

# C++ facade (what an ORB-SLAM3 build compiles) + its GPU test program
FACADE_TEST := tests/cpp/build/facade_test
facade_test: $(FACADE_TEST)
FACADE_SRC := orbslam3lib_amd/facade/ORBextractor.cc orbslam3lib_amd/facade/LynxHardwareAccelerator.cc
FACADE_HDR := include/orbslam3/ORBextractor.h include/orbslam3/cv_shim.h \
	include/orbslam3/LynxHardwareAcceleration/LynxHardwareAccelerator.h
$(FACADE_TEST): tests/cpp/facade_test.cpp $(FACADE_SRC) $(FACADE_HDR) $(LIB)
	@mkdir -p tests/cpp/build
	$(CXX) -O2 -std=c++17 -Wall -o $@ tests/cpp/facade_test.cpp $(FACADE_SRC) -pthread \
		-L orbslam3lib_amd -lorbgpu -Wl,-rpath,'$$ORIGIN/../../../orbslam3lib_amd' -Wl,-rpath-link,/opt/rocm/lib -ldl

# plain-C consumer of the IDL-shaped entry point (gcc, C99)
IDL_TEST := tests/c/build/idl_test
idl_test: $(IDL_TEST)
$(IDL_TEST): tests/c/idl_test.c include/orbgpu.h $(LIB)
	@mkdir -p tests/c/build
	$(CC) -O2 -std=c99 -Wall -Iinclude -o $@ tests/c/idl_test.c -L orbslam3lib_amd -lorbgpu \
		-Wl,-rpath,'$$ORIGIN/../../../orbslam3lib_amd' -Wl,-rpath-link,/opt/rocm/lib

clean:
	rm -f $(LIB) $(LIBOBJ)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean facade_test idl_test
