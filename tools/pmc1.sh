cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_INST[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|SQ_LDS[A-Z_0-9]*\|TCC_HIT[A-Z_0-9]*\|TCC_MISS[A-Z_0-9]*\|FETCH_SIZE\|WRITE_SIZE\|SQ_BUSY[A-Z_0-9]*\|SQ_WAVE[A-Z_0-9]*\|SQ_ACTIVE[A-Z_0-9]*" gpurun_out/counters.txt | sort -u > gpurun_out/counter_names.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1
echo rc=$?
