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

.PHONY: all lib oracle ref examples clean
all: lib oracle examples

lib: $(LIB)

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/ort_kernel.o: $(SRC)/ort_kernel.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/gpu_build.o: $(SRC)/gpu_build.hip $(SRC)/gpu_build.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -Wno-unused-result -c $< -o $@

$(OBJ)/group.o: $(SRC)/group.hip $(SRC)/group_map.h $(SRC)/ort_internal.h include/ort.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJS) $(HIP_OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl -Wl,-soname,libort.so

examples: build/ort_main

build/ort_main: examples/main.cpp $(LIB) $(HDRS)
	$(CXX) -O2 -std=c++17 -I$(SRC) -o $@ examples/main.cpp -L$(dir $(LIB)) -lort -Wl,-rpath,'$$ORIGIN/../$(dir $(LIB))'

oracle:
	$(MAKE) -C oracle all

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean
