# Build everything in-tree (the .so files travel to the GPU box with the
# repo snapshot; they are git-ignored).
#   make            HIP library (gfx950) + oracle (test infrastructure)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -Wall

LIB = hiccl_amd/libhiccl_reduce.so

PROBE = tools/libhbm_probe.so

all: $(LIB) $(PROBE) cpp oracle

$(PROBE): tools/hbm_probe.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

# The atomic optimizer rewrites the one-lane unit-ticket grab into a
# wave-reduction whose result is read back at once (s_waitcnt vmcnt(0) at the
# top of every unit); without it the wait lands after the unit's last add.
LIBFLAGS = -mllvm -amdgpu-atomic-optimizer-strategy=None

$(LIB): hiccl_amd/csrc/reduce.hip include/hiccl_reduce.h
	$(HIPCC) $(HIPFLAGS) $(LIBFLAGS) -o $@ $<

# oracle/_ref/collectives_main_hip links the HIP library: build it first
oracle: $(LIB)
	$(MAKE) -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# ---- C++ surface (include/hiccl.h): drivers and test tools -----------------
MPI_INC ?= /opt/conda/include
MPI_LIB ?= /opt/conda/lib
CXX ?= g++
CXXFLAGS = -std=c++17 -O2 -Wall -Wno-unused-function -Iinclude -I$(MPI_INC)
MPI_LINK = $(MPI_LIB)/libmpi.so -Wl,-rpath,/usr/lib/x86_64-linux-gnu:$(MPI_LIB)
# the XCCL level runs on RCCL point-to-point (include/hiccl/transport.h)
HIP_HOST = -D__HIP_PLATFORM_AMD__ -DHICCL_WITH_RCCL -I/opt/rocm/include
HIP_LINK = -Lhiccl_amd -lhiccl_reduce -Wl,-rpath,'$$ORIGIN/../hiccl_amd' -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
ABI_LINK = -Lhiccl_amd -lhiccl_reduce -Wl,-rpath,'$$ORIGIN/../hiccl_amd' -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
HDRS = include/hiccl.h $(wildcard include/hiccl/*.h) include/hiccl_reduce.h hiccl_amd/csrc/compose.h

CPP_BINS = build/plan_dump build/collectives_host build/collectives_host_f32 build/collectives_hip build/collectives_hip_f32 \
           build/readme_example_host build/readme_example_hip build/abi_c build/ipc_reuse build/sync_wait_probe

cpp: $(CPP_BINS)

build/plan_dump: tests/cpp/plan_dump.cpp $(HDRS)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -o $@ $< $(MPI_LINK)

build/collectives_host: hiccl_amd/csrc/collectives.cpp $(HDRS)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -fopenmp -DHICCL_PORT_HOST -o $@ $< $(MPI_LINK)

build/collectives_host_f32: hiccl_amd/csrc/collectives.cpp $(HDRS)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -fopenmp -DHICCL_PORT_HOST -DHICCL_DRIVER_FLOAT -o $@ $< $(MPI_LINK)

build/collectives_hip: hiccl_amd/csrc/collectives.cpp $(HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) $(HIP_HOST) -o $@ $< $(HIP_LINK) $(MPI_LINK)

build/collectives_hip_f32: hiccl_amd/csrc/collectives.cpp $(HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) $(HIP_HOST) -DHICCL_DRIVER_FLOAT -o $@ $< $(HIP_LINK) $(MPI_LINK)

build/readme_example_host: hiccl_amd/csrc/readme_example.cpp $(HDRS)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -fopenmp -DHICCL_PORT_HOST -o $@ $< $(MPI_LINK)

build/readme_example_hip: hiccl_amd/csrc/readme_example.cpp $(HDRS) $(LIB)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) $(HIP_HOST) -o $@ $< $(HIP_LINK) $(MPI_LINK)

# two-process reproducer of the IPC close/reopen behaviour (tests/test_ipc_reuse_gpu.py)
build/ipc_reuse: tests/cpp/ipc_reuse.cpp include/hiccl_reduce.h $(LIB)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< $(ABI_LINK) $(MPI_LINK)

# host wait after a C5-step launch, from C++ (tools/sync_wait_probe.cpp)
build/sync_wait_probe: tools/sync_wait_probe.cpp include/hiccl_reduce.h $(LIB)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< $(ABI_LINK)

# plain C99 client of the C ABI (the header must stay C)
build/abi_c: tests/cpp/abi_c.c include/hiccl_reduce.h $(LIB)
	@mkdir -p build
	gcc -std=c99 -pedantic -Wall -Wextra -Werror -Iinclude -o $@ $< $(ABI_LINK)

.PHONY: cpp
