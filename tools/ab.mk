# A/B and diagnostic variant builds of libtcsc_amd.so (not part of the
# product build).  Run from the package directory so the product Makefile's
# variables and object rules apply:
#
#   make -C sparse-matrix-multiplication-benchmark_amd -f ../tools/ab.mk lib/abl/libtcsc_amd_pfs0.so
#
# Every target writes under lib/abl, lib/geo or lib/wid, which .gpurunignore
# keeps out of GPU pushes; an A/B session lists the builds it needs in its
# own gpurun command (tools/ab.sh) after removing them from .gpurunignore.
include Makefile

# Timing-only ablation builds of the gather loop (tools/gen_gather_asm.py):
# lib/abl/libtcsc_amd_abl<N>.so, loaded via TCSC_AMD_LIB=... (results wrong).
ABLS := 1 3 4 5 6
ablation: $(foreach a,$(ABLS),lib/abl/libtcsc_amd_abl$(a).so)

lib/abl/libtcsc_amd_abl%.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_ABLATION=$* -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k$*.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# diagnostic build: s_memtime stamps of the chunk loop's waits written into Y
lib/abl/libtcsc_amd_stamps.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_STAMPS -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_stamps.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_stamps.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# diagnostic build: per-interval, per-wave timeline of the chunk loop written into Y (tools/trace.py)
lib/abl/libtcsc_amd_trace.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_TRACE -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_trace.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_trace.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# staging variants (A/B): lib/abl/libtcsc_amd_dma<waves>_<early>.so
lib/abl/libtcsc_amd_dma%.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_DMA_WAVES=$(word 1,$(subst _, ,$*)) -DTCSC_DMA_EARLY=$(word 2,$(subst _, ,$*)) -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_dma$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_dma$*.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# longest-stream-first wave priority (TCSC_PRIO = batch threshold of prio 1)
lib/abl/libtcsc_amd_prio%.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_PRIO=$* -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_prio$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_prio$*.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# the same without the X staging (gather cost alone): lib/abl/libtcsc_amd_abl<N>_nd.so
ablation-nodma: $(foreach a,0 1 3 4 5,lib/abl/libtcsc_amd_abl$(a)_nd.so)

lib/abl/libtcsc_amd_abl%_nd.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_ABLATION=$* -DTCSC_NODMA -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k$*_nd.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k$*_nd.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# Gather-geometry variants: lib/geo/libtcsc_amd_w<W>_cw<CW>_b<B>_c<CAP>_tk<TK>_nb<NBUF>[_d<D>].so
# (waves per workgroup, columns per wave, batch, SGPR stream capacity, K rows
# per chunk, LDS ring buffers, batches in flight; the VGPR budget per wave follows from W:
# 512 / (W/4)).  Plan and kernel are built from the same constants.
GEOS := w16_cw16_b4_c16_tk48_nb3 w16_cw16_b4_c32_tk48_nb3 w12_cw24_b4_c32_tk48_nb3 w16_cw16_b4_c24_tk64_nb2
geometry: $(foreach g,$(GEOS),lib/geo/libtcsc_amd_$(g).so)

geo_f = $(patsubst $(2)%,%,$(word $(3),$(subst _, ,$(1))))
geo_budget = $(shell echo $$(( 512 / ($(call geo_f,$(1),w,1) / 4) / 8 * 8 )))
geo_defs = -DTCSC_WAVES=$(call geo_f,$(1),w,1) -DTCSC_CW=$(call geo_f,$(1),cw,2) -DTCSC_BATCH=$(call geo_f,$(1),b,3) \
           -DTCSC_TK=$(call geo_f,$(1),tk,5) -DTCSC_NBUF=$(call geo_f,$(1),nb,6)

$(OBJ)/geo/gather_%.inc: ../tools/gen_gather_asm.py
	@mkdir -p $(OBJ)/geo
	python3 ../tools/gen_gather_asm.py --cw $(call geo_f,$*,cw,2) --batch $(call geo_f,$*,b,3) \
	    --cap $(call geo_f,$*,c,4) --budget $(call geo_budget,$*) --depth $(or $(call geo_f,$*,d,7),1) --touch $(or $(patsubst t%,%,$(filter t%,$(word 8,$(subst _, ,$*)))),0) -o $@ > /dev/null

lib/geo/libtcsc_amd_%.so: $(OBJ)/geo/gather_%.inc $(SRC)/tcsc_kernels.hip $(SRC)/tcsc_api.cpp $(HDRS) $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o
	@mkdir -p lib/geo
	$(HIPCC) $(HIPFLAGS) $(call geo_defs,$*) -DTCSC_GATHER_INC='"$(abspath $(OBJ)/geo/gather_$*.inc)"' \
	    -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/geo/k_$*.o
	$(HIPCC) $(HIPFLAGS) $(call geo_defs,$*) -c $(SRC)/tcsc_api.cpp -o $(OBJ)/geo/a_$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/geo/k_$*.o $(OBJ)/geo/a_$*.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

.SECONDARY:
.PHONY: ablation ablation-nodma geometry
# Per-rank column widths (TCSC_WIDTHS, tcsc_internal.h): lib/wid/libtcsc_amd_wd<A>_<B>_<C>_<D>.so,
# waves of age rank r own <r-th> columns each, accumulators for the widest.
comma := ,
wid_cw = $(shell printf '%s\n' $(subst _, ,$(1)) | sort -n | tail -n 1)
$(OBJ)/wid/gather_cw%.inc: ../tools/gen_gather_asm.py
	@mkdir -p $(OBJ)/wid
	python3 ../tools/gen_gather_asm.py --cw $* -o $@ > /dev/null

.SECONDEXPANSION:
lib/wid/libtcsc_amd_wd%.so: $(OBJ)/wid/gather_cw$$(call wid_cw,$$*).inc $(SRC)/tcsc_kernels.hip $(SRC)/tcsc_api.cpp $(HDRS) $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o
	@mkdir -p lib/wid $(OBJ)/wid
	$(HIPCC) $(HIPFLAGS) -DTCSC_CW=$(call wid_cw,$*) -DTCSC_WIDTHS=$(subst _,$(comma),$*) \
	    -DTCSC_GATHER_INC='"$(abspath $(OBJ)/wid/gather_cw$(call wid_cw,$*).inc)"' -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/wid/k_$*.o
	$(HIPCC) $(HIPFLAGS) -DTCSC_CW=$(call wid_cw,$*) -DTCSC_WIDTHS=$(subst _,$(comma),$*) -c $(SRC)/tcsc_api.cpp -o $(OBJ)/wid/a_$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/wid/k_$*.o $(OBJ)/wid/a_$*.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas

# stream-prefetch on/off (A/B): lib/abl/libtcsc_amd_pfs<0|1>.so (distance and width: TCSC_PF_DIST / TCSC_PF_LINES)
lib/abl/libtcsc_amd_pfs%.so: $(SRC)/tcsc_kernels.hip $(SRC)/tcsc_api.cpp $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_PF_S=$* -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_pfs$*.o
	$(HIPCC) $(HIPFLAGS) -DTCSC_PF_S=$* -c $(SRC)/tcsc_api.cpp -o $(OBJ)/abl/a_pfs$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_pfs$*.o $(OBJ)/abl/a_pfs$*.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas -Wl,-rpath,$(ROCM)/lib

# k_fused (the persistent gather with in-kernel X^T production, round 4) left the
# library in round 5: the kernel, its launcher and its A/B variants are at commit
# 815156e (csrc/tcsc_kernels.hip k_fused, tools/ab.mk lib/abl/libtcsc_amd_f<v>.so).

# 4-byte entry cost proxy: the generated loop rebuilds the +-1
# multiplier from a sign bit with 2 SALU per entry (gen_gather_asm.py --sgn 1);
# results unchanged.  lib/abl/libtcsc_amd_sgn1.so
$(OBJ)/abl/gather_sgn%.inc: ../tools/gen_gather_asm.py
	@mkdir -p $(OBJ)/abl
	python3 ../tools/gen_gather_asm.py --sgn $* -o $@ > /dev/null

lib/abl/libtcsc_amd_sgn%.so: $(OBJ)/abl/gather_sgn%.inc $(SRC)/tcsc_kernels.hip $(SRC)/tcsc_api.cpp $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS)
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_GATHER_INC='"$(abspath $(OBJ)/abl/gather_sgn$*.inc)"' -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_sgn$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_sgn$*.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas -Wl,-rpath,$(ROCM)/lib

# split-K combine slab loads: nontemporal (default) or cached (rnt0)
lib/abl/libtcsc_amd_rnt%.so: $(SRC)/tcsc_kernels.hip $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o $(HDRS) $(SRC)/gather_asm.inc
	@mkdir -p lib/abl $(OBJ)/abl
	$(HIPCC) $(HIPFLAGS) -DTCSC_REDUCE_NT=$* -c $(SRC)/tcsc_kernels.hip -o $(OBJ)/abl/k_rnt$*.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)/abl/k_rnt$*.o $(OBJ)/tcsc_api.o $(OBJ)/tcsc_mfma.o $(OBJ)/tcsc_small.o $(OBJ)/tcsc_format.o $(OBJ)/tcsc_cxx_abi.o $(OBJ)/bcsr_kernels.o $(OBJ)/bcsr_api.o -lpthread -L$(ROCM)/lib -lrocblas -Wl,-rpath,$(ROCM)/lib

# Direct X staging (A/B, round 5, DESIGN.md §4 k_transpose): the variant and its target
# lib/abl/libtcsc_amd_xs1.so are at commit b07f36f (measured slower, removed).
