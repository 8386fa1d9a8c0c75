# Builds libtic.so (gfx950 HIP kernels + C-ABI runtime) in-tree so it travels with the
# repo snapshot to the GPU box.  `make -j8` here cross-compiles without a GPU.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := tf_image_compression_amd/csrc
BUILD    := build
LIB      := tf_image_compression_amd/libtic.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -I$(CSRC)
KERNELS  := conv_s1 conv_s2 conv_t2 conv_rgb conv_chain image_ops
OBJS     := $(addprefix $(BUILD)/,$(addsuffix .o,$(KERNELS))) $(BUILD)/tic_runtime.o $(BUILD)/range_coder.o \
            $(BUILD)/host_util.o
HDRS     := $(wildcard $(CSRC)/*.h) include/tic.h

all: $(LIB)

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/tic_runtime.o: $(CSRC)/tic_runtime.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/range_coder.o: $(CSRC)/range_coder.cpp include/tic.h | $(BUILD)
	g++ -O2 -std=c++17 -fPIC -Wall -Iinclude -c $< -o $@

$(BUILD)/host_util.o: $(CSRC)/host_util.cpp include/tic.h | $(BUILD)
	g++ -O2 -std=c++17 -fPIC -Wall -Iinclude -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-rpath,/opt/rocm/lib

$(BUILD):
	mkdir -p $(BUILD)

# Host sanitizer build (CPU only): the host C++ that parses user input (range coder,
# CRC-32C of checkpoint bytes) under AddressSanitizer + UBSan, driven by a fuzz harness.
ASAN_BIN := $(BUILD)/host_fuzz_asan
asan: $(ASAN_BIN)
	$(ASAN_BIN) $(BUILD)

$(ASAN_BIN): tests/native/host_fuzz.cpp $(CSRC)/range_coder.cpp $(CSRC)/host_util.cpp include/tic.h | $(BUILD)
	g++ -O1 -g -std=c++17 -Wall -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all \
	    -Iinclude -o $@ tests/native/host_fuzz.cpp $(CSRC)/range_coder.cpp $(CSRC)/host_util.cpp

clean:
	rm -rf $(BUILD) $(LIB)

.PHONY: all clean asan
