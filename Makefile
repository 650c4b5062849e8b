# liborbgpu.so: the MI355X (gfx950) ORB front-end.  `make` here or __graft_entry__.build().
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := orbslam3lib_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
# MFMA accumulators in VGPRs (k_knn2_mfma reads every result: no v_accvgpr copies)
DEVFLAGS := -mllvm -amdgpu-mfma-vgpr-form
LIB := orbslam3lib_amd/liborbgpu.so
HDRS := $(wildcard $(CSRC)/*.h) include/orbgpu.h

all: $(LIB) oracle facade_test

$(LIB): $(CSRC)/orb_kernels.hip $(CSRC)/orb_stereo.hip $(CSRC)/orb_frame.hip $(CSRC)/orb_runtime.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -shared -o $@ $(CSRC)/orb_kernels.hip $(CSRC)/orb_stereo.hip $(CSRC)/orb_frame.hip $(CSRC)/orb_runtime.cpp

oracle:
	$(MAKE) -s -C oracle

# C++ facade (what an ORB-SLAM3 build compiles) + its GPU test program
FACADE_TEST := tests/cpp/build/facade_test
facade_test: $(FACADE_TEST)
$(FACADE_TEST): tests/cpp/facade_test.cpp orbslam3lib_amd/facade/ORBextractor.cc include/orbslam3/ORBextractor.h include/orbslam3/cv_shim.h $(LIB)
	@mkdir -p tests/cpp/build
	$(CXX) -O2 -std=c++17 -o $@ tests/cpp/facade_test.cpp orbslam3lib_amd/facade/ORBextractor.cc \
		-L orbslam3lib_amd -lorbgpu -Wl,-rpath,'$$ORIGIN/../../../orbslam3lib_amd' -Wl,-rpath-link,/opt/rocm/lib -ldl

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean facade_test
