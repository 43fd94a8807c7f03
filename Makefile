# Builds the product library octreeraytracer_amd/lib/libort.so (host scene stage + gfx950
# kernel + C ABI) and the test-only oracle (oracle/liboracle.so, oracle/_ref/ref_octree).
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
SRC := octreeraytracer_amd/csrc
OBJ := build/obj
LIB := octreeraytracer_amd/lib/libort.so
CXXFLAGS := -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -Wall -Wno-unused-parameter

HOST_SRCS := octree.cpp scene.cpp host_abi.cpp layout.cpp raytracer.cpp
HOST_OBJS := $(addprefix $(OBJ)/,$(HOST_SRCS:.cpp=.o))
HIP_OBJS := $(OBJ)/ort_kernel.o $(OBJ)/gpu_build.o $(OBJ)/group.o
HDRS := $(wildcard $(SRC)/*.h) $(SRC)/prebuilt_scene.inc include/ort.h include/ort_math.h

# The analysis library (test/analysis surface: ort_debug_* host emulation and walk statistics,
# ORT_OPT_DEBUG_FLAGS) -- the same sources with -DORT_ANALYSIS=1; the CPU suite and tools/
# load it, the product library does not carry it.
ALIB := octreeraytracer_amd/lib/libort_analysis.so
AOBJ := build/obj_analysis

.PHONY: all lib analysis oracle ref examples san clean
all: lib analysis oracle examples

lib: $(LIB)

analysis: $(ALIB)

$(AOBJ)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(AOBJ)
	$(HIPCC) $(HIPFLAGS) -DORT_ANALYSIS=1 -c $< -o $@

$(ALIB): $(HOST_OBJS) $(AOBJ)/ort_kernel.o $(OBJ)/gpu_build.o $(AOBJ)/group.o
	@mkdir -p $(dir $(ALIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -Wl,-soname,libort_analysis.so -Wl,-Bsymbolic

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJ)/ort_kernel.o: $(SRC)/ort_kernel.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/gpu_build.o: $(SRC)/gpu_build.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -Wno-unused-result -c $< -o $@

$(OBJ)/group.o: $(SRC)/group.hip $(SRC)/group_map.h $(SRC)/ort_internal.h include/ort.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJS) $(HIP_OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -Wl,-soname,libort.so

examples: build/ort_main build/stats_row

build/stats_row: tests/cpp/stats_row.cpp $(LIB) $(HDRS)
	$(CXX) -O2 -std=c++17 -I$(SRC) -o $@ tests/cpp/stats_row.cpp -L$(dir $(LIB)) -lort -Wl,-rpath,'$$ORIGIN/../$(dir $(LIB))'

build/ort_main: examples/main.cpp $(LIB) $(HDRS)
	$(CXX) -O2 -std=c++17 -I$(SRC) -o $@ examples/main.cpp -L$(dir $(LIB)) -lort -Wl,-rpath,'$$ORIGIN/../$(dir $(LIB))'

oracle:
	$(MAKE) -C oracle all

# Host AddressSanitizer + UndefinedBehaviorSanitizer build (CPU only; GPU sanitizers are not
# available): every host object -- scene stage, octree builder, layout compilers, host ABI,
# the kernel's per-pixel code compiled for the host, the group row map, the oracle -- built
# with clang and instrumented, linked into build/san/san_check (tests/cpp/san_check.cpp),
# which renders small frames through the emulation and the oracle and compares bits.
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
SANOBJ := build/san
CLANGXX := /opt/rocm/bin/amdclang++
CLANG := /opt/rocm/bin/amdclang
SAN_HOST := $(addprefix $(SANOBJ)/,$(HOST_SRCS:.cpp=.o))
SAN_HIP := $(SANOBJ)/ort_kernel.o $(SANOBJ)/gpu_build.o $(SANOBJ)/group.o
HIP_SAN := $(foreach f,address undefined,-Xarch_host -fsanitize=$(f)) -Xarch_host -fno-sanitize-recover=undefined

san: build/san/san_check
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 ./build/san/san_check

$(SANOBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(SANOBJ)
	$(CLANGXX) $(SAN) -std=c++17 -ffp-contract=off -fno-fast-math -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(SANOBJ)/%.o: $(SRC)/%.hip $(HDRS) $(SRC)/gpu_build.h $(SRC)/group_map.h
	@mkdir -p $(SANOBJ)
	$(HIPCC) -O1 -g -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-result -DORT_ANALYSIS=1 $(HIP_SAN) -c $< -o $@

$(SANOBJ)/ort_oracle.o: oracle/ort_oracle.c oracle/ort_oracle.h include/ort_math.h
	@mkdir -p $(SANOBJ)
	$(CLANG) $(SAN) -std=c11 -ffp-contract=off -fno-fast-math -c $< -o $@

$(SANOBJ)/san_check.o: tests/cpp/san_check.cpp $(HDRS) oracle/ort_oracle.h
	@mkdir -p $(SANOBJ)
	$(CLANGXX) $(SAN) -std=c++17 -I$(SRC) -Ioracle -c $< -o $@

build/san/san_check: $(SANOBJ)/san_check.o $(SAN_HOST) $(SAN_HIP) $(SANOBJ)/ort_oracle.o
	$(HIPCC) --offload-arch=$(ARCH) $(SAN) -o $@ $^ -ldl

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf build $(LIB) $(ALIB)
	$(MAKE) -C oracle clean
