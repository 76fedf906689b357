# Build for the MI355X (gfx950) newsched block-execution path. No cmake/meson needed:
#   libnsh_hip.so    HIP kernels + C-ABI (include/nsh_hip.h)        -- hipcc, gfx950 only
#   libnewsched.so   C++17 host runtime + blocks + GPU domain         -- g++, links libnsh_hip
#   tests/cpp/*      C++ behaviour tests (restated reference gtests)  -- g++
#   oracle/_build    CPU oracle (test infrastructure)                 -- gcc
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
LIBDIR   := newsched_amd/lib
OBJDIR   := build/obj
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Wall -Wno-unused-function
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -pthread \
            -Iinclude -Inewsched_amd/runtime/include -Inewsched_amd/schedulers/include \
            -Inewsched_amd/blocklib/include

HIP_SRC  := $(wildcard newsched_amd/csrc/*.hip)
HIP_OBJ  := $(patsubst newsched_amd/csrc/%.hip,$(OBJDIR)/hip/%.o,$(HIP_SRC))
RT_SRC   := $(wildcard newsched_amd/runtime/lib/*.cpp) $(wildcard newsched_amd/schedulers/lib/*.cpp) \
            $(wildcard newsched_amd/blocklib/lib/*.cpp) $(wildcard newsched_amd/capi/*.cpp)
RT_OBJ   := $(patsubst newsched_amd/%.cpp,$(OBJDIR)/rt/%.o,$(RT_SRC))
RT_HDR   := $(shell find newsched_amd/runtime/include newsched_amd/schedulers/include newsched_amd/blocklib/include -name '*.hpp' 2>/dev/null)
TEST_SRC := $(wildcard tests/cpp/*.cpp)
TEST_BIN := $(patsubst tests/cpp/%.cpp,build/tests/%,$(TEST_SRC))
TOOL_SRC := $(wildcard tools/*.cpp)
TOOL_BIN := $(patsubst tools/%.cpp,build/tools/%,$(TOOL_SRC))

all: hip runtime tests tools oracle
hip: $(LIBDIR)/libnsh_hip.so
runtime: $(LIBDIR)/libnewsched.so
tests: $(TEST_BIN) build/tests/libfake_rccl.so
tools: $(TOOL_BIN)
oracle:
	$(MAKE) -C oracle

$(OBJDIR)/hip/%.o: newsched_amd/csrc/%.hip $(wildcard newsched_amd/csrc/*.hpp) include/nsh_hip.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libnsh_hip.so: $(HIP_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJ)

$(OBJDIR)/rt/%.o: newsched_amd/%.cpp $(RT_HDR) include/nsh_hip.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIBDIR)/libnewsched.so: $(RT_OBJ) $(LIBDIR)/libnsh_hip.so
	$(CXX) -shared -fPIC -pthread -o $@ $(RT_OBJ) -L$(LIBDIR) -lnsh_hip -Wl,-rpath,'$$ORIGIN'

build/tests/%: tests/cpp/%.cpp $(LIBDIR)/libnewsched.so $(wildcard tests/cpp/*.hpp)
	@mkdir -p build/tests
	$(CXX) $(CXXFLAGS) -Itests/cpp -o $@ $< -L$(LIBDIR) -lnewsched -lnsh_hip -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

# RCCL test double for the remote edge's rccl transport (rendezvous semantics on device rings,
# tests/test_remote_edge.py, tests/test_bench.py)
build/tests/libfake_rccl.so: tests/cpp/fake_rccl.hip
	@mkdir -p build/tests
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -fPIC -shared -Wall -pthread -o $@ $<

build/tools/%: tools/%.cpp $(LIBDIR)/libnewsched.so
	@mkdir -p build/tools
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(LIBDIR) -lnewsched -lnsh_hip -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

clean:
	rm -rf build $(LIBDIR)
	$(MAKE) -C oracle clean

.PHONY: all hip runtime tests tools oracle clean
