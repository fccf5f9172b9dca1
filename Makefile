# Build everything in-tree (the .so files travel to the GPU box with the
# repo snapshot; they are git-ignored).
#   make            HIP library (gfx950) + oracle (test infrastructure)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -Wall

LIB = hiccl_amd/libhiccl_reduce.so

all: $(LIB) oracle

$(LIB): hiccl_amd/csrc/reduce.hip include/hiccl_reduce.h
	$(HIPCC) $(HIPFLAGS) -o $@ $<

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
