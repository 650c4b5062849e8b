# liborbgpu.so: the MI355X (gfx950) ORB front-end.  `make` here or __graft_entry__.build().
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := orbslam3lib_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
LIB := orbslam3lib_amd/liborbgpu.so
HDRS := $(wildcard $(CSRC)/*.h) include/orbgpu.h

all: $(LIB) oracle

$(LIB): $(CSRC)/orb_kernels.hip $(CSRC)/orb_runtime.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/orb_kernels.hip $(CSRC)/orb_runtime.cpp

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
