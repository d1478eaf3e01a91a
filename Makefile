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
ifeq ($(KTRACE),1)   # per-phase shader-clock trace of K1 and the log fire (GWO_KTRACE=1 at run time; diagnostics)
HIPFLAGS += -DGWO_KTRACE
endif
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

# JNI shim for the Java GpuWindowOperator (java/): built only where a JDK provides jni.h (none in this image).
JAVA_HOME ?= /usr/lib/jvm/default-java
JNI_LIB := flink_amd/libgwo_jni.so
jni: $(LIB)
	@if [ -f "$(JAVA_HOME)/include/jni.h" ]; then \
	  $(CXX_HOST:g++=gcc) -O2 -fPIC -shared -Wall -I$(JAVA_HOME)/include -I$(JAVA_HOME)/include/linux -Iinclude \
	    jni/gwo_jni.c -o $(JNI_LIB) -Lflink_amd -lgwo -Wl,-rpath,'$$ORIGIN'; \
	  echo "built $(JNI_LIB)"; \
	else echo "jni: no $(JAVA_HOME)/include/jni.h -- skipped (set JAVA_HOME to a JDK)"; fi
# Java classes (needs javac and the Flink jars on FLINK_CLASSPATH)
java-classes:
	@if command -v javac >/dev/null 2>&1 && [ -n "$(FLINK_CLASSPATH)" ]; then \
	  mkdir -p build/java && javac -d build/java -cp "$(FLINK_CLASSPATH)" $$(find java -name '*.java'); \
	else echo "java-classes: javac or FLINK_CLASSPATH missing -- skipped"; fi
.PHONY: jni java-classes

# Access-pattern microbenchmark of the table layout; not part of the library.
tools/micro_table: tools/micro_table.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
tools: tools/micro_table
.PHONY: tools
