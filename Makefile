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

# LEGACY=1 adds the superseded FIR matrix-core kernels (k_fir_mfma2/5/7/9, k_fir_casc2: A/B runs
# and their parity tests, pytest marker `legacy`); the default library leaves them out
LEGACY   ?= 0
HIP_SRC  := $(wildcard newsched_amd/csrc/*.hip)
ifeq ($(LEGACY),1)
HIP_SRC  += newsched_amd/csrc/legacy/nsh_fir_legacy.hip
endif
HIP_OBJ  := $(patsubst newsched_amd/csrc/%.hip,$(OBJDIR)/hip/%.o,$(HIP_SRC))
LEGACY_STAMP := $(OBJDIR)/legacy_$(LEGACY).stamp
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

# relink when LEGACY changes (the object list shrinks without any object getting newer)
$(LEGACY_STAMP):
	@mkdir -p $(OBJDIR)
	@rm -f $(OBJDIR)/legacy_*.stamp
	@touch $@

$(LIBDIR)/libnsh_hip.so: $(HIP_OBJ) $(LEGACY_STAMP)
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

# RCCL test double for the remote edge's rccl transport on host rings (tests/test_remote_edge.py)
build/tests/libfake_rccl.so: tests/cpp/fake_rccl.c
	@mkdir -p build/tests
	$(CC) -O2 -std=gnu11 -fPIC -shared -Wall -Wextra -pthread -o $@ $< -ldl

build/tools/%: tools/%.cpp $(LIBDIR)/libnewsched.so
	@mkdir -p build/tools
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(LIBDIR) -lnewsched -lnsh_hip -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

clean:
	rm -rf build $(LIBDIR)
	$(MAKE) -C oracle clean

.PHONY: all hip runtime tests tools oracle clean
