# Build of libmatvec_gpu.so (HIP + RCCL, gfx950), the three drop-in executables and the
# CPU oracle. Everything is written in-tree so the built .so/binaries travel with the repo
# snapshot to the GPU box.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
ROCM     ?= /opt/rocm
PKG      := matvec_mpi_multiplier_amd
CSRC     := $(PKG)/csrc
BUILD    := build
LIB      := $(PKG)/libmatvec_gpu.so
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result -munsafe-fp-atomics
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
LDLIBS   := -L$(ROCM)/lib -lamdhip64 -lrccl -lpthread -Wl,-rpath,$(ROCM)/lib

HIP_SRCS := $(CSRC)/gemv.hip
CXX_SRCS := $(CSRC)/host.cpp $(CSRC)/engine.cpp $(CSRC)/textio.cpp
HDRS     := $(CSRC)/common.h include/matvec_gpu.h
OBJS     := $(BUILD)/gemv.o $(BUILD)/host.o $(BUILD)/engine.o $(BUILD)/textio.o
APPS     := bin/multiplier_rowwise bin/multiplier_colwise bin/multiplier_blockwise

EXAMPLES := bin/rowwise_binding

all: $(LIB) $(APPS) $(EXAMPLES) oracle

examples: $(EXAMPLES)

bin/rowwise_binding: examples/rowwise_binding.c $(LIB) include/matvec_gpu.h | $(BUILD)
	gcc -O2 -std=c99 -D_POSIX_C_SOURCE=199309L -Wall -Wextra $< -o $@ -L$(PKG) -lmatvec_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)'


$(BUILD):
	mkdir -p $(BUILD) bin

$(BUILD)/gemv.o: $(CSRC)/gemv.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(CXXFLAGS) -x c++ -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@ $(LDLIBS)

bin/multiplier_rowwise: apps/multiplier_main.cpp $(LIB) include/matvec_gpu.h | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=0 $< -o $@ -L$(PKG) -lmatvec_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)' -lpthread
bin/multiplier_colwise: apps/multiplier_main.cpp $(LIB) include/matvec_gpu.h | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=1 $< -o $@ -L$(PKG) -lmatvec_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)' -lpthread
bin/multiplier_blockwise: apps/multiplier_main.cpp $(LIB) include/matvec_gpu.h | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=2 $< -o $@ -L$(PKG) -lmatvec_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)' -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB) $(APPS) $(EXAMPLES)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle examples
