# Build the MI355X engine (gfx950) and the C oracle.  No cmake needed.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
SRC = kmamiz_amd/csrc/kmz_kernels.hip kmamiz_amd/csrc/kmz_part.hip kmamiz_amd/csrc/kmz_join.hip kmamiz_amd/csrc/kmz_chain.hip kmamiz_amd/csrc/kmz_api.hip kmamiz_amd/csrc/kmz_tail.hip kmamiz_amd/csrc/kmz_guard.hip kmamiz_amd/csrc/kmz_shard.hip kmamiz_amd/csrc/kmz_order.hip kmamiz_amd/csrc/kmz_json.hip kmamiz_amd/csrc/kmz_fuse.hip kmamiz_amd/csrc/kmz_walk.hip
HDR = include/kmz.h kmamiz_amd/csrc/kmz_common.h kmamiz_amd/csrc/kmz_joinw.h kmamiz_amd/csrc/kmz_chainw.h kmamiz_amd/csrc/kmz_walkw.h kmamiz_amd/csrc/kmz_synth.h kmamiz_amd/csrc/kmz_kernels.h
OBJ = build/kmz_kernels.o build/kmz_part.o build/kmz_join.o build/kmz_chain.o build/kmz_api.o build/kmz_ingest.o build/kmz_tail.o build/kmz_guard.o build/kmz_shard.o build/kmz_order.o build/kmz_json.o build/kmz_fuse.o build/kmz_walk.o

all: kmamiz_amd/libkmz.so oracle addon

build/%.o: kmamiz_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only sources (the Zipkin JSON ingest)
build/%.o: kmamiz_amd/csrc/%.cpp include/kmz.h
	@mkdir -p build
	g++ -O3 -std=c++17 -fPIC -Wall -pthread -c $< -o $@

kmamiz_amd/libkmz.so: $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $@ $(OBJ)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build kmamiz_amd/libkmz.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# Node N-API addon (seam 1 of SURVEY.md 8b); built when node headers exist
NODE_INC ?= /usr/include/node
js/kmz.node: js/kmz_napi.c include/kmz.h kmamiz_amd/libkmz.so
	gcc -O2 -fPIC -shared -Wall -I$(NODE_INC) -o $@ js/kmz_napi.c -Lkmamiz_amd -lkmz -Wl,-rpath,'$$ORIGIN/../kmamiz_amd'

addon:
	@if [ -f $(NODE_INC)/node_api.h ]; then $(MAKE) js/kmz.node; else echo "no node headers: addon skipped"; fi
.PHONY: addon
