# Ablation timings (kernel_ms = gather + reduce, prepared X) for one config: full, no gather, no DMA, skeleton
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=sparse-matrix-multiplication-benchmark_amd/lib
A="--steps 20 --warmup 10 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs ${BENCH_ARGS:-}"
for a in 0 5 6 5_nd 0; do
  lib=$P/libtcsc_amd.so; [ $a != 0 ] && lib=$P/abl/libtcsc_amd_abl$a.so
  V=""; [ $a != 0 ] && V="--no-validate"
  TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py $A $V > gpurun_out/ablc.json 2> gpurun_out/ablc.err
  rc=$?; [ $rc -ne 0 ] && { echo "abl $a rc=$rc"; tail -3 gpurun_out/ablc.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/ablc.json')); r=d['roofline']; print('abl $a', round(r['kernel_ms']*1e3,1), 'us gather+reduce;', round(r['transpose_ms']*1e3,1), 'us transpose;', round(d['ms_per_step']*1e3,1), 'us/step')"
done
