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

HIP_SRCS := $(CSRC)/gemv.hip $(CSRC)/gemv_exact.hip
CXX_SRCS := $(CSRC)/host.cpp $(CSRC)/engine.cpp $(CSRC)/textio.cpp
HDRS     := $(CSRC)/common.h $(CSRC)/lds_dma.h include/matvec_gpu.h
OBJS     := $(BUILD)/gemv.o $(BUILD)/gemv_exact.o $(BUILD)/host.o $(BUILD)/engine.o $(BUILD)/textio.o
APPS     := bin/multiplier_rowwise bin/multiplier_colwise bin/multiplier_blockwise

# The executables' launcher (apps/launch.h): over MPI when one is installed (the image's MPICH
# under /opt/conda, or MPI_HOME=...), so `mpiexec -n P bin/multiplier_<alg>` runs P ranks; else
# single-process only. MPI stays inside bin/libmvg_launch.so and its own run path.
MPI_HOME ?= /opt/conda
ifneq ($(wildcard $(MPI_HOME)/include/mpi.h),)
LAUNCH_SRC  := apps/launch_mpi.c
LAUNCH_LIBS := -I$(MPI_HOME)/include -L$(MPI_HOME)/lib -lmpi -Wl,-rpath,$(MPI_HOME)/lib
else
LAUNCH_SRC  := apps/launch_none.c
LAUNCH_LIBS :=
endif
LAUNCH   := bin/libmvg_launch.so
APP_LINK := -L$(PKG) -lmatvec_gpu -Lbin -lmvg_launch -Wl,-rpath,'$$ORIGIN/../$(PKG)' -Wl,-rpath,'$$ORIGIN' -lpthread

EXAMPLES := bin/rowwise_binding

all: $(LIB) $(LAUNCH) $(APPS) $(EXAMPLES) oracle

examples: $(EXAMPLES)

bin/rowwise_binding: examples/rowwise_binding.c $(LIB) include/matvec_gpu.h | $(BUILD)
	gcc -O2 -std=c99 -D_POSIX_C_SOURCE=199309L -Wall -Wextra $< -o $@ -L$(PKG) -lmatvec_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)'


$(BUILD):
	mkdir -p $(BUILD) bin

$(BUILD)/gemv.o: $(CSRC)/gemv.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the bit-exact kernels must never fuse a*b + c (the reference rounds the product first)
$(BUILD)/gemv_exact.o: $(CSRC)/gemv_exact.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -ffp-contract=off -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(CXXFLAGS) -x c++ -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@ $(LDLIBS)

$(LAUNCH): $(LAUNCH_SRC) apps/launch.h | $(BUILD)
	gcc -O2 -std=c99 -fPIC -shared -Wall -Wextra $(LAUNCH_SRC) -o $@ $(LAUNCH_LIBS)

APP_DEPS := apps/multiplier_main.cpp apps/launch.h $(LIB) $(LAUNCH) include/matvec_gpu.h
bin/multiplier_rowwise: $(APP_DEPS) | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=0 $< -o $@ $(APP_LINK)
bin/multiplier_colwise: $(APP_DEPS) | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=1 $< -o $@ $(APP_LINK)
bin/multiplier_blockwise: $(APP_DEPS) | $(BUILD)
	g++ -O2 -std=c++17 -Wall -DMVG_APP_ALG=2 $< -o $@ $(APP_LINK)

oracle:
	$(MAKE) -C oracle

# ---- the host code under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU only
# (SURVEY §5): the library's host translation units (planner, engine, text loader) and the
# oracle, built with the ROCm clang (host code; the kernels' objects are linked unchanged), then
# the CPU tests that drive them (tools/asan_tests.sh). Nothing here runs on a GPU.
ASAN_DIR := $(BUILD)/asan
CLANGXX  := $(ROCM)/lib/llvm/bin/clang++
CLANGC   := $(ROCM)/lib/llvm/bin/clang
SANFLAGS := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
ASAN_OBJS := $(ASAN_DIR)/host.o $(ASAN_DIR)/engine.o $(ASAN_DIR)/textio.o

asan: $(ASAN_DIR)/libmatvec_gpu.so $(ASAN_DIR)/liboracle.so

$(ASAN_DIR):
	mkdir -p $(ASAN_DIR)

$(ASAN_DIR)/%.o: $(CSRC)/%.cpp $(HDRS) | $(ASAN_DIR)
	$(CLANGXX) -std=c++17 -fPIC -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include $(SANFLAGS) -c $< -o $@

$(ASAN_DIR)/libmatvec_gpu.so: $(ASAN_OBJS) $(BUILD)/gemv.o $(BUILD)/gemv_exact.o
	$(CLANGXX) -shared -fPIC -shared-libasan $(SANFLAGS) $(BUILD)/gemv.o $(BUILD)/gemv_exact.o $(ASAN_OBJS) -o $@ $(LDLIBS)

$(ASAN_DIR)/liboracle.so: oracle/cpu_ref.c oracle/cpu_ref.h | $(ASAN_DIR)
	$(CLANGC) -std=c11 -fPIC -shared -shared-libasan -ffp-contract=off -pthread $(SANFLAGS) $< -o $@

clean:
	rm -rf $(BUILD) $(LIB) $(LAUNCH) $(APPS) $(EXAMPLES)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle examples asan
