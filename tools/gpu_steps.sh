#!/bin/bash
# GPU steps by name, for gpurun:  TAG=r03a tools/gpu_steps.sh cfg4 inv cfg5factor pmcbench
# Each step runs under its own time limit; a failure, abort or timeout ends the call (no retries, no
# further GPU step).  Logs and profiles under gpurun_out/$TAG/.
set -o pipefail
O=gpurun_out/${TAG:-r03}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  # progress line every 60 s while the step runs (each step is bounded by its own time limit)
  ( while sleep 60; do echo "   $name running $(date +%T), log $(wc -l < "$O/$name.log") lines"; done ) &
  local hb=$!
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  tail -n "${TAILN:-6}" "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    gpu)        step gputests 1100 $PYT -m gpu tests ;;
    gpunoab)    step gputests 1100 $PYT -m gpu tests -k "not edge_sweep_matches_abi9" ;;
    edgeab)     # test failures (rc 1) do not end the call; a timeout, abort or crash does
      ( TAILN=30 step edgeab 300 ${PYT/-x/--maxfail 20} -s tests/test_gpu_ns_velocity.py -k edge_sweep_matches_abi9 )
      rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    gpurest)    step gpurest 900 $PYT -m gpu tests/test_gpu_krylov.py tests/test_gpu_ns_velocity.py \
                  tests/test_gpu_partition.py tests/test_gpu_solvers.py tests/test_gpu_boussinesq.py tests/test_gpu_cfg4.py ;;
    nsbenchab)  step nsbenchab 300 python tools/nsbench.py --kernels band,tile ;;
    cfg4)       step cfg4 300 $PYT -s tests/test_gpu_cfg4.py ;;
    nsapply)    step nsapply 300 $PYT tests/test_gpu_ns_apply.py ;;
    velocity)   step velocity 600 $PYT tests/test_gpu_ns_velocity.py ;;
    mfmatest)   step mfmatest 600 $PYT tests/test_gpu_apply.py ;;
    mfmapmc)    tools/pmc_run.sh "$O/pmc_mfma64" -- python tools/kbench.py --meshes 8:64 --reps 200 --algo 2 || exit 1 ;;
    batchedinv) step batchedinv 300 $PYT tests/test_batched_inverse.py tests/test_gpu_dense_inverse.py ;;
    smoke)      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)      step bench 600 python bench.py ;;
    benchgloo)  # the N > 1 bench path (strip partition, interface exchange, max-over-ranks timing) rehearsed with
                # several ranks on one GPU over gloo (RCCL needs one GPU per rank); all-reduce and p2p exchanges
      for nr in 2 4; do for ex in allreduce p2p; do
        step benchgloo_${nr}_$ex 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $nr \
          --master-addr 127.0.0.1 --master-port 2962$nr bench.py --gpus $nr --steps 20 --warmup 5 \
          --dist-backend gloo --exchange $ex --cpu-seconds 0 --extra-steps 20
      done; done ;;
    benchdrv)   step benchdrv 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;   # the driver's command
    pmccd64)    tools/pmc_run.sh "$O/pmc_cd64" -- python tools/kbench.py --meshes 8:64 --reps 200 || exit 1 ;;
    inv)        step inv 300 python tools/inv_repro.py ;;
    nsbench)    step nsbench 300 python tools/nsbench.py ;;
    pivot)      step pivot 300 python tools/pivot_probe.py ;;
    gemvprobe)  step gemvprobe 300 python tools/gemv_probe.py ;;
    dist)       step dist 900 $PYT tests/test_gpu_dist.py -k "not cfg5_element_partitioned_ns_update" ;;
    distcfg5)   step distcfg5 720 ${PYT/--timeout 300/--timeout 680} -s tests/test_gpu_dist.py -k cfg5_element_partitioned_ns_update ;;
    cfg5factor) SEM_PROFILE_FACTOR=1 step cfg5factor 900 python tools/cfg5_ns_probe.py --update 0 ;;
    cfg5factor_inv) SEM_PIVOT_INV=inv SEM_PROFILE_FACTOR=1 step cfg5factor_inv 900 python tools/cfg5_ns_probe.py --update 0 ;;
    cfg5ns)     SEM_PROFILE_FACTOR=1 step cfg5ns 900 python tools/cfg5_ns_probe.py ;;
    pmcbench)
      tools/pmc_run.sh "$O/pmc_cal" -- python tools/kbench.py --dss 1024 || exit 1
      tools/pmc_run.sh "$O/pmc_cd64" -- python tools/kbench.py --meshes 8:64 --reps 200 || exit 1
      tools/pmc_run.sh "$O/pmc_cd1024" -- python tools/kbench.py --meshes 8:1024 --reps 20 || exit 1
      tools/pmc_run.sh "$O/pmc_mfma64" -- python tools/kbench.py --meshes 8:64 --reps 200 --algo 2 || exit 1
      tools/pmc_run.sh "$O/pmc_dot2" -- python tools/sweep_bench.py || exit 1 ;;
    pmcns)
      tools/pmc_run.sh "$O/pmc_ns48" -- python tools/nsbench.py --meshes 8:48 --reps 100 || exit 1
      tools/pmc_run.sh "$O/pmc_ns128" -- python tools/nsbench.py --meshes 12:128 --reps 20 || exit 1
      tools/pmc_run.sh "$O/pmc_vel48" -- python tools/velocity_bench.py --ne 48 --P 8 --configs nested:cr --reps 20 \
        || exit 1 ;;
    pmcns128)
      tools/pmc_run.sh "$O/pmc_ns128" -- python tools/nsbench.py --meshes 12:128 --reps 20 || exit 1 ;;
    cfg5trace)
      step cfg5trace 900 rocprofv3 --kernel-trace --stats -d "$O/cfg5trace" -o trace --output-format csv -- \
        python tools/cfg5_ns_probe.py --update 0
      python tools/pmc_compact.py "$O/cfg5trace" && python tools/prof_summary.py "$O/cfg5trace" "" > "$O/cfg5trace/prof_summary.txt" ;;
    vsolve)     step vsolve 600 python tools/vsolve_probe.py --out "$O/vsolve.json" ;;
    sweepab)    # interface sweep A/B: one-ended against two-ended block Thomas, one process each, alternated
      for rep in 1 2; do for f in single twisted; do
        SEM_SWEEP_FORM=$f TAILN=1 step sweepab_${f}_$rep 300 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 \
          --out "$O/sweepab_${f}_$rep.json"
      done; done ;;
    edgetw)     # two-ended edge sweep (ABI 12) against the one-ended one (EDGE_THOMAS = 2): cfg2-size and 128^2 P=12
      SEM_EDGE_TWISTED=1 TAILN=2 step edgetw_48 300 python tools/vsolve_probe.py --ne 48 --P 8 --ab-edge 0 --ab-back 0 --ab-oneended 1 \
        --solves 50 --out "$O/edgetw_48.json"
      SEM_EDGE_TWISTED=1 TAILN=2 step edgetw_128 600 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 --ab-oneended 1 \
        --out "$O/edgetw_128.json" ;;
    gemvcpol)   # streaming GEMV operator loads plain (2) against non-temporal (0, the default): shapes alone, then the
                # cfg5 velocity solve, one process per setting, alternated (bitwise-identical results)
      for rep in 1 2; do for c in 2 0; do
        SEM_GEMV_CPOL=$c TAILN=3 step gemvcpol_${c}_$rep 300 python tools/gemv_shapes.py
        SEM_GEMV_CPOL=$c TAILN=1 step vsolvecpol_${c}_$rep 300 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 \
          --solves 30 --out "$O/vsolvecpol_${c}_$rep.json"
      done; done ;;
    gemvshape)  # streaming GEMV rows per workgroup x loads in flight (SEM_GEMV_SHAPE 0-4; bitwise-identical results):
                # the bitwise test, then the operator shapes and the cfg5 velocity solve, one process per variant
      SEM_TEST_GEMV_SHAPES=8 step gemvshapetest 300 $PYT tests/test_gpu_ns_velocity.py -k "shapes_and_load_policy"
      for rep in 1 2; do for v in ${GEMV_SHAPES:-0 3 5 6 7}; do
        SEM_GEMV_SHAPE=$v TAILN=3 step gemvshape_${v}_$rep 300 python tools/gemv_shapes.py
        SEM_GEMV_SHAPE=$v TAILN=1 step vsolveshape_${v}_$rep 300 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 \
          --solves 30 --out "$O/vsolveshape_${v}_$rep.json"
      done; done ;;
    cpolab)     # non-temporal loads (1) against plain (0), one process per setting, alternated (bitwise-identical results):
                # the Krylov basis passes (sweep_bench at the 64^2 CD size and at cfg4's Ra = 1e6 block solve) and the
                # nested solve's element step (the cfg5 velocity solve)
      for rep in 1 2; do for c in 0 1; do
        SEM_BASIS_CPOL=$c TAILN=4 step sweepcpol_${c}_$rep 300 python tools/sweep_bench.py
        SEM_BASIS_CPOL=$c TAILN=2 step schurcpol_${c}_$rep 300 python tools/schur_ab.py --precond mass \
          --out "$O/schurcpol_${c}_$rep.jsonl"
        SEM_COND_CPOL=$c TAILN=1 step condcpol_${c}_$rep 300 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 \
          --solves 30 --out "$O/condcpol_${c}_$rep.json"
      done; done ;;
    vsolveab)   # interface-sweep GEMV A/B: the library's streaming GEMV (default) against rocBLAS, one process each
      SEM_SWEEP_GEMV=torch TAILN=2 step vsolve_rocblas 600 python tools/vsolve_probe.py --ab-edge 0 --out "$O/vsolve_rocblas.json"
      TAILN=2 step vsolve_hip 600 python tools/vsolve_probe.py --ab-edge 1 --out "$O/vsolve_hip.json" ;;
    vsolvetrace)  # kernel trace of one factor + the A/B + 20 solves; FETCH_SIZE / WRITE_SIZE passes of their own
      step vsolvetrace 900 rocprofv3 --kernel-trace --stats -d "$O/vsolvetrace" -o trace --output-format csv -- \
        python tools/vsolve_probe.py --out "$O/vsolvetrace.json"
      TAILN=40 step vsolve_window 120 python tools/trace_window.py "$O/vsolvetrace" 20 cond_fwd_kernel 2 \
        --save "$O/vsolvetrace/window_20_solves.csv"
      find "$O/vsolvetrace" -name "*kernel_trace.csv" -delete   # the window and --stats stay; the full trace is ~100 MB
      step vsolve_fetch 600 timeout -s KILL 580 rocprofv3 --pmc FETCH_SIZE -d "$O/vsolve_pmc1" -o pmc --output-format csv -- \
        python tools/vsolve_probe.py --ab-edge 0
      step vsolve_write 600 timeout -s KILL 580 rocprofv3 --pmc WRITE_SIZE -d "$O/vsolve_pmc2" -o pmc --output-format csv -- \
        python tools/vsolve_probe.py --ab-edge 0
      python tools/pmc_compact.py "$O/vsolve_pmc1" && python tools/pmc_compact.py "$O/vsolve_pmc2" && du -sh "$O" ;;
    vsolvetr)   # kernel trace of one factor + 20 solves of the default path (no A/B, no PMC passes)
      step vsolvetr 600 rocprofv3 --kernel-trace --stats -d "$O/vsolvetr" -o trace --output-format csv -- \
        python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 --out "$O/vsolvetr.json"
      TAILN=40 step vsolvetr_window 120 python tools/trace_window.py "$O/vsolvetr" 20 cond_fwd_kernel 1 \
        --save "$O/vsolvetr/window_20_solves.csv"
      find "$O/vsolvetr" -name "*kernel_trace.csv" -delete ;;
    vsolvepmc)  # FETCH_SIZE / WRITE_SIZE of the default velocity solve (one pass each, no tracing domains)
      step vsolvepmc_fetch 600 timeout -s KILL 580 rocprofv3 --pmc FETCH_SIZE -d "$O/vsolvepmc1" -o pmc --output-format csv -- \
        python tools/vsolve_probe.py --ab-edge 0 --ab-back 0
      step vsolvepmc_write 600 timeout -s KILL 580 rocprofv3 --pmc WRITE_SIZE -d "$O/vsolvepmc2" -o pmc --output-format csv -- \
        python tools/vsolve_probe.py --ab-edge 0 --ab-back 0
      python tools/pmc_compact.py "$O/vsolvepmc1" && python tools/pmc_compact.py "$O/vsolvepmc2" ;;
    bandlab)    # cfg2 latency anatomy: diagnostic ablations (sem_amd/lib_diag) and the trivial-kernel floor
      step dispatch 120 tools/dispatch_bench
      for kp in 0 -1; do for d in 0 16 32 48 112; do
        SEM_LIBDIR=$PWD/sem_amd/lib_diag SEM_ALLOW_DIAG=1 SEM_BAND_KP=$kp SEM_DIAG=$d \
          step bandlab_kp${kp}_d$d 120 python tools/kbench.py --meshes 8:64 --reps 1000
      done; done ;;
    stamps)     # cfg2 per-wave phase stamps and per-tile realtime start/end (diagnostic build, struct-argument kernel)
      for rep in 1 2; do
        SEM_LIBDIR=$PWD/sem_amd/lib_diag SEM_ALLOW_DIAG=1 SEM_BAND_KP=0 SEM_DIAG=8 SEM_DIAG_BUF=auto TAILN=30 \
          step stamps_$rep 120 python tools/kbench.py --meshes 8:64 --stamps --nstamps 6 --stride 16 \
          --roles X:0-1,Y:2-3 --tiles-x 65 --tiles-y 9
      done ;;
    kbench)     TAILN=4 step kbench 300 python tools/kbench.py --meshes 8:64,12:128,8:1024 --reps 1000 ;;
    bandtests)  step bandtests 600 $PYT tests/test_gpu_apply.py tests/test_gpu_partition.py ;;
    orderab)    # band tile order A/B: full tiles first (0) against the round-3 order (1), alternated, one process each
      for rep in 1 2 3; do for o in 0 1; do
        SEM_BAND_ORDER=$o TAILN=2 step orderab_${o}_$rep 120 python tools/kbench.py --meshes 8:64,8:256 --reps 2000
      done; done ;;
    schurab)    TAILN=4 step schurab 900 python tools/schur_ab.py --out "$O/schur_ab.jsonl" ;;
    schurpipe)  # device GMRES pipelined step A/B at cfg4's Ra = 1e6 block solve, one process each, alternated
      for rep in 1 2; do for pp in 0 1; do
        SEM_GMRES_PIPELINE=$pp TAILN=2 step schurpipe_${pp}_$rep 300 python tools/schur_ab.py --precond mass \
          --out "$O/schurpipe_${pp}_$rep.jsonl"
      done; done ;;
    schurmass)  TAILN=4 step schurmass 300 python tools/schur_ab.py --precond mass --out "$O/schur_mass.jsonl" ;;
    krylovgpu)  step krylovgpu 300 $PYT tests/test_gpu_krylov.py tests/test_gpu_cfg4.py ;;
    cfg5solve)  step cfg5solve 1000 python -u tools/bous_cfg5_solve.py --continuation 1e3 --Ra 1e4 \
                  --out "$O/cfg5_ra1e4.json" ;;
    cfg4part)   # the element-partitioned coupled solve end to end at cfg4's size (48^2, P=8): 4 ranks on one GPU, gloo
      step cfg4part 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29613 tools/bous_cfg5_solve.py --backend gloo --ne 48 --P 8 --Ra 1e3 --out "$O/cfg4_part4_ra1e3.json" ;;
    cfg4whole)  step cfg4whole 300 python tools/bous_cfg5_solve.py --ne 48 --P 8 --Ra 1e3 --out "$O/cfg4_whole_ra1e3.json" ;;
    cfg5part)   # rehearsal of cfg5's element-partitioned coupled solve: 4 ranks on one GPU over gloo, Ra = 1e3 from rest
      step cfg5part 1080 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29611 tools/bous_cfg5_solve.py --backend gloo --Ra 1e3 --out "$O/cfg5_part4_ra1e3.json" ;;
    benchtrace)
      step bench 600 python bench.py
      step benchtrace 600 rocprofv3 --kernel-trace --stats -d "$O/benchtrace" -o trace --output-format csv -- \
        python bench.py --cpu-seconds 0 ;;
    bandab)     # every band-kernel variant on the HBM mesh and cfg2 (one process per knob value: read once)
      step bandab_floor 300 python tools/kbench.py --meshes 8:1024 --reps 100 --floor
      for t in 0 1 2 3 4 5 6 7 8 9; do
        SEM_BAND_TILE=$t step bandab_t$t 300 python tools/kbench.py --meshes 8:64,8:1024 --reps 200
      done
      for w in 512 2048 4096; do
        SEM_BAND_TILE=8 SEM_MARCH_WG=$w step bandab_m$w 300 python tools/kbench.py --meshes 8:1024 --reps 200
      done
      for c in 5 1 4 257 260; do
        SEM_BAND_CPOL=$c step bandab_c$c 300 python tools/kbench.py --meshes 8:1024 --reps 200
      done ;;
    krylovdist) step krylovdist 900 $PYT tests/test_gpu_krylov.py tests/test_gpu_dist.py ;;
    stripprof)  # where the partitioned Schur matvec's time goes (gloo rehearsal, 4 ranks) and
                # one cfg5 strip as rank r of 8 alone on the GPU (loopback collectives), beside the whole-mesh matvec
      step stripprof48 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29631 tools/strip_profile.py --mode rehearsal --ne 48 --P 8 --reps 5 --iters 40 \
        --out "$O/strip_rehearsal48.jsonl"
      step stripsolo128 900 python tools/strip_profile.py --mode solo --ne 128 --P 12 --G 8 --ranks 0,3 --reps 10 \
        --whole 1 --out "$O/strip_solo128.jsonl" ;;
    stripsolo)
      step stripsolo128 900 python tools/strip_profile.py --mode solo --ne 128 --P 12 --G 8 --ranks 0,3 --reps 10 \
        --whole 1 --out "$O/strip_solo128.jsonl" ;;
    edgeprint)  TAILN=40 step edgeprint 300 $PYT -s tests/test_gpu_ns_velocity.py -k edge_sweep ;;
    ghostab)    # VERDICT r4 item 7, the upper bound of folding the ghost tiles away: the 512 full tiles alone (diagnostic
                # bit 128, wrong closing line / column) against all 585 tiles, alternated, in the driver's shape (one
                # 20-apply graph) and amortised (1000-apply graph); then the SQ counter passes of both
      for rep in 1 2 3; do for d in 0 128; do
        SEM_LIBDIR=$PWD/sem_amd/lib_diag SEM_ALLOW_DIAG=1 SEM_DIAG=$d TAILN=2 step ghostab_d${d}_r20_$rep 120 \
          python tools/kbench.py --meshes 8:64 --reps 20
        SEM_LIBDIR=$PWD/sem_amd/lib_diag SEM_ALLOW_DIAG=1 SEM_DIAG=$d TAILN=2 step ghostab_d${d}_r1000_$rep 120 \
          python tools/kbench.py --meshes 8:64 --reps 1000
      done; done
      for d in 0 128; do
        SEM_LIBDIR=$PWD/sem_amd/lib_diag SEM_ALLOW_DIAG=1 SEM_DIAG=$d tools/pmc_run.sh "$O/pmc_ghost_d$d" -- \
          python tools/kbench.py --meshes 8:64 --reps 200 || exit 1
      done ;;
    stripsolocr)  # the round-4 reduced solve (block CR replicated on every rank) in the same solo measurement
      SEM_STRIP_REDUCED=cr step stripsolocr 900 python tools/strip_profile.py --mode solo --ne 128 --P 12 --G 8 --ranks 3 \
        --reps 10 --whole 0 --out "$O/strip_solo128_cr.jsonl" ;;
    stripsolotrace)  # kernel trace of one simulated cfg5 rank of 8 (factor + matvecs), per-kernel split of the strip solve
      step stripsolotrace 600 rocprofv3 --kernel-trace --stats -d "$O/stripsolotrace" -o trace --output-format csv -- \
        python tools/strip_profile.py --mode solo --ne 128 --P 12 --G 8 --ranks 3 --reps 10 --whole 0
      find "$O/stripsolotrace" -name "*kernel_trace.csv" -size +20M -delete ;;
    cfg4a)      # BASELINE cfg4 end to end, part 1: Ra 1e3 -> 1e4 -> 1e5 -> 3e5 from rest, checkpointed
      step cfg4a 1150 python -u tools/bous_solve.py --ne 48 --P 8 --continuation 1e3,1e4,1e5 --Ra 3e5 --iprint 2 \
        --ckpt "$O/ckpt" --out "$O/cfg4_to3e5.json" ;;
    cfg4b)      # part 2: Ra = 1e6 from the Ra = 3e5 state cfg4a wrote to $O/ckpt (ckpt/ is ignored by git
                # and gpurun, so the start state must come from this session's own cfg4a step); its sha256 goes
                # into the step log for the record
      sha256sum "$O/ckpt/bous_48_300000.npy" | tee -a "$O/cfg4_provenance.txt"
      step cfg4b 1150 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --x0 "$O/ckpt/bous_48_300000.npy" --iprint 2 \
        --ckpt "$O/ckpt" --out "$O/cfg4_ra1e6.json" ;;
    cfg4c)      # part 3 (if part 2 hit its limit): Ra = 1e6 resumed from part 2's last Newton checkpoint in $O/ckpt
      sha256sum "$O/ckpt/bous_48_1e+06_newton.npy" | tee -a "$O/cfg4_provenance.txt"
      step cfg4c 1150 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --x0 "$O/ckpt/bous_48_1e+06_newton.npy" \
        --resume 1 --iprint 2 --ckpt "$O/ckpt" --out "$O/cfg4_ra1e6_resumed.json" ;;
    bmfma)      # band-form MFMA kernel (round 5): parity, then A/B against the band VALU kernel and the element-block
                # MFMA kernel of rounds 1-4 (SEM_MFMA_TILE=3), and the counter passes of the new kernel at cfg2
      step bmfmatests 900 $PYT tests/test_gpu_apply.py tests/test_gpu_partition.py
      for rep in 1 2; do
        TAILN=4 step bmfma_ab_new_$rep 300 python tools/kbench.py --meshes 8:64,12:128,8:1024 --reps 500 --algo 2
        SEM_MFMA_TILE=3 TAILN=4 step bmfma_ab_eb_$rep 300 python tools/kbench.py --meshes 8:64,12:128,8:1024 --reps 500 --algo 2
        TAILN=4 step bmfma_ab_band_$rep 300 python tools/kbench.py --meshes 8:64,12:128,8:1024 --reps 500 --algo 0
      done
      tools/pmc_run.sh "$O/pmc_bmfma64" -- python tools/kbench.py --meshes 8:64 --reps 200 --algo 2 || exit 1 ;;
    bmfmapmc)   TAILN=4 step bmfma_apply 300 $PYT tests/test_gpu_apply.py tests/test_gpu_partition.py
      TAILN=4 step bmfma_kb 300 python tools/kbench.py --meshes 8:64,12:128,8:1024 --reps 500 --algo 2
      tools/pmc_run.sh "$O/pmc_bmfma64" -- python tools/kbench.py --meshes 8:64 --reps 200 --algo 2 || exit 1 ;;
    gemvshapes) TAILN=4 step gemvshapes 300 python tools/gemv_shapes.py ;;
    stripprof128)
      step stripprof128 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29632 tools/strip_profile.py --mode rehearsal --ne 128 --P 12 --reps 3 --iters 10 \
        --out "$O/strip_rehearsal128.jsonl" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps ok"
