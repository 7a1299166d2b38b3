# mipipe native build: HIP kernels (gfx950) + C++ runtime -> libmipipe.so, plus the C++ tools.
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PKG       := distributed-llm-pipeline_amd
LIBDIR    := $(PKG)/lib
BINDIR    := $(PKG)/bin
BUILD     := build
CXXFLAGS  := -std=c++17 -O3 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-result \
             -I$(ROCM)/include -Icsrc/runtime
# `make PROBES=1 BUILD=build_probes LIBDIR=...`: a separate library with the timing-probe knobs
# (GEMM3_PROBE, ATTN_PROBE), which skip work and give wrong results; the default build has none
ifeq ($(PROBES),1)
CXXFLAGS  += -DMIPIPE_TIMING_PROBES
endif
HIPFLAGS  := $(CXXFLAGS) --offload-arch=$(ARCH) -munsafe-fp-atomics
LDFLAGS   := -L$(ROCM)/lib -lrccl -lpthread -Wl,-rpath,$(ROCM)/lib

KSRC := $(wildcard csrc/kernels/*.hip)
RSRC := $(wildcard csrc/runtime/*.cpp)
KOBJ := $(patsubst csrc/kernels/%.hip,$(BUILD)/k_%.o,$(KSRC))
ROBJ := $(patsubst csrc/runtime/%.cpp,$(BUILD)/r_%.o,$(RSRC))
HDRS := $(wildcard csrc/kernels/*.h csrc/runtime/*.h)

all: $(LIBDIR)/libmipipe.so tools

$(BUILD):
	mkdir -p $(BUILD) $(LIBDIR) $(BINDIR)

$(BUILD)/k_%.o: csrc/kernels/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/r_%.o: csrc/runtime/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(CXXFLAGS) --offload-arch=$(ARCH) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(LIBDIR)/libmipipe.so: $(KOBJ) $(ROBJ) | $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(KOBJ) $(ROBJ) $(LDFLAGS)

TOOLS := $(patsubst csrc/tools/%.cpp,$(BINDIR)/%,$(wildcard csrc/tools/*.cpp))
tools: $(TOOLS)

$(BINDIR)/%: csrc/tools/%.cpp $(LIBDIR)/libmipipe.so $(HDRS) $(wildcard csrc/tools/*.h)
	$(HIPCC) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -Icsrc/tools $< $(wildcard csrc/tools/*_impl.cpp) -o $@ \
	  -L$(LIBDIR) -lmipipe -Wl,-rpath,'$$ORIGIN/../lib' $(LDFLAGS)

# Host-only ASan/UBSan build of the untrusted-input parsers (GGUF, tokenizer, JSON) for
# tests/test_sanitize.py; no GPU code involved
SAN_SRC := csrc/tools/fuzz_host.cpp csrc/runtime/gguf.cpp csrc/runtime/json.cpp csrc/runtime/model.cpp \
           csrc/runtime/tokenizer.cpp csrc/runtime/log.cpp
$(BUILD)/fuzz_host_asan: $(SAN_SRC) $(HDRS) | $(BUILD)
	g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
	  -Icsrc/runtime $(SAN_SRC) -o $@
sanitize: $(BUILD)/fuzz_host_asan

clean:
	rm -rf $(BUILD) $(LIBDIR)/libmipipe.so $(TOOLS)

.PHONY: all tools clean sanitize
