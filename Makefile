# Builds the product library (HIP, gfx950) and the CPU oracle (test infra).
# No cmake: plain hipcc / gcc.  `python -c "import __graft_entry__ as g; g.build()"` runs this.
HIPCC  ?= /opt/rocm/bin/hipcc
ARCH   ?= gfx950
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
BUILD  := build
CSRC   := lz4mt_amd/csrc
LIB    := lz4mt_amd/liblz4mt_amd.so
OBJS   := $(BUILD)/lz4mt_kernels.o $(BUILD)/lz4mt_engine.o $(BUILD)/lz4mt_frame.o $(BUILD)/lz4mt_io.o
HDRS   := $(CSRC)/lz4mt_device.h $(CSRC)/lz4mt_host.h include/lz4mt.h include/lz4mt_hip.h include/lz4mt_io.h

all: $(LIB) oracle

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
