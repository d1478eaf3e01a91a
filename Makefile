# Builds the C-ABI library flink_amd/libgwo.so for gfx950 (kernels: hipcc; host runtime: g++).
# `python -c "import __graft_entry__ as g; g.build()"` drives this Makefile.
ROCM ?= /opt/rocm
ARCH ?= gfx950
HIPCC ?= $(ROCM)/bin/hipcc
CXX_HOST ?= g++
BUILD := build/obj
LIB := flink_amd/libgwo.so

HIP_SRCS := $(wildcard flink_amd/csrc/*.hip)
CPP_SRCS := $(wildcard flink_amd/csrc/*.cpp)
HIP_OBJS := $(patsubst flink_amd/csrc/%.hip,$(BUILD)/%.hip.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst flink_amd/csrc/%.cpp,$(BUILD)/%.cpp.o,$(CPP_SRCS))
HDRS := $(wildcard flink_amd/csrc/*.h) include/gwo.h

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
CXXFLAGS := -O2 -std=c++17 -fPIC -Wall -Wno-unused-function -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include

all: $(LIB)

# gwo_log.hip: no atomic optimizer -- it turns the fire's single-lane row reservation into a
# wave scan + readfirstlane that waits for the atomic's round trip on the spot.
$(BUILD)/gwo_log.hip.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None

$(BUILD)/%.hip.o: flink_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.cpp.o: flink_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(CXX_HOST) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,$(ROCM)/lib

clean:
	rm -rf build $(LIB)

.PHONY: all clean

# Access-pattern microbenchmark of the table layout; not part of the library.
tools/micro_table: tools/micro_table.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
tools: tools/micro_table
.PHONY: tools
