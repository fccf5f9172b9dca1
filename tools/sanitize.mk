# Host-port builds under AddressSanitizer + UndefinedBehaviorSanitizer (g++,
# CPU only: the C++ surface's schedule, factorization and host reduction).
# Used by tests/test_host_sanitize.py; never built for or run on a GPU box.
#   make -f tools/sanitize.mk
CXX ?= g++
MPI_INC ?= /opt/conda/include
MPI_LIB ?= /opt/conda/lib
SANFLAGS = -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined \
           -Wall -Wno-unused-function -Iinclude -I$(MPI_INC)
MPI_LINK = $(MPI_LIB)/libmpi.so -Wl,-rpath,/usr/lib/x86_64-linux-gnu:$(MPI_LIB)
HDRS = include/hiccl.h $(wildcard include/hiccl/*.h)

all: build/san/collectives_host_f32 build/san/plan_dump

build/san/collectives_host_f32: hiccl_amd/csrc/collectives.cpp $(HDRS)
	@mkdir -p build/san
	$(CXX) $(SANFLAGS) -fopenmp -DHICCL_PORT_HOST -DHICCL_DRIVER_FLOAT -o $@ $< $(MPI_LINK)

build/san/plan_dump: tests/cpp/plan_dump.cpp $(HDRS)
	@mkdir -p build/san
	$(CXX) $(SANFLAGS) -o $@ $< $(MPI_LINK)

.PHONY: all
