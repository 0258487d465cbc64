#!/bin/bash
# Run GPU steps on the gpurun box; stop at the first crash-class exit status
# (fault/abort/segv/timeout), keep going after ordinary test failures (rc 1).
#   tools/gpu_session.sh smoke tests bench prof pmc
# Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out

step() {  # name, timeout-seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a $OUT/session.log
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "crash-class exit ($rc) in $name: stopping" | tee -a $OUT/session.log
    exit $rc
  fi
  return 0
}

for s in "$@"; do
  case $s in
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 1080 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    testsnew) step pytest_new 1200 python -u -m pytest tests/test_gpu_delivery.py tests/test_gpu_fullsize.py tests/test_gpu_peer_push.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    testslog) step pytest_log 600 python -u -m pytest tests/test_gpu_log_layout.py tests/test_gpu_peer_group.py tests/test_gpu_bench_protocol.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    testsuni) step pytest_uni 600 python -u -m pytest tests/test_gpu_log_layout.py tests/test_gpu_uniform_rows.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    gm_um) step gm_um4 600 python tools/group_model.py --workload c4 --ranks 4 --kinds targets --target-option uni_merge=2 --json $OUT/group_model_c4_um4.json && \
           step gm_um8 600 python tools/group_model.py --workload c4 --ranks 8 --kinds targets --target-option uni_merge=4 --json $OUT/group_model_c4_um8.json && \
           step gm_um8t16 600 python tools/group_model.py --workload c4 --ranks 8 --kinds targets --target-option tiles_per_wave=16 --json $OUT/group_model_c4_t16.json ;;
    wbprobe) step wbprobe 600 python tools/wb_probe.py --json $OUT/wb_probe.json ;;
    ab_c2emit) step ab_c2emit 600 bash -c 'for i in 1 2 3; do for v in default late emit2 emit2late; do echo "== $v"; if [ $v = default ]; then python tools/fuse_probe.py | head -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py | head -1; fi; done; done' ;;
    gm_t16) step gm_t16_c4 600 python tools/group_model.py --workload c4 --ranks 4,8 --kinds targets --target-option tiles_per_wave=16 --json $OUT/gm_t16_c4.json && \
            step gm_t16_c4p 600 python tools/group_model.py --workload c4p --ranks 4,8 --kinds targets --target-option tiles_per_wave=16 --json $OUT/gm_t16_c4p.json && \
            step gm_t16_c4pb 600 python tools/group_model.py --workload c4pb --ranks 4,8 --kinds targets --target-option tiles_per_wave=16 --json $OUT/gm_t16_c4pb.json ;;
    ab_c2e) step ab_c2e 600 bash -c 'for i in 1 2 3; do for v in default emit2 late emit2late; do echo "== $v"; if [ $v = default ]; then python tools/fuse_probe.py --fuse 16 --repeat 15; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py --fuse 16 --repeat 15; fi; done; done' ;;
    ab_c5tpw) step ab_c5tpw 600 bash -c 'for i in 1 2; do for t in 8 16; do echo "== tpw $t"; python tools/round_probe.py --workload c5 --option tiles_per_wave=$t | tail -1; done; done' ;;
    gm_td) for w in c4 c4p c4pb; do
             step gm_td0_$w 600 python tools/group_model.py --workload $w --ranks 2,4,8 --kinds targets --target-option tile_draw=0 --json $OUT/gm_td0_$w.json || exit $?
             step gm_td16_$w 600 python tools/group_model.py --workload $w --ranks 2,4,8 --kinds targets --target-option tiles_per_wave=16 --json $OUT/gm_td16_$w.json || exit $?
           done ;;
    ab_c5td) step ab_c5td 600 bash -c 'for i in 1 2; do for o in "tile_draw=0" "tile_draw=1" "tile_draw=1 --option tiles_per_wave=16"; do echo "== $o"; python tools/round_probe.py --workload c5 --option $o | tail -1; done; done' ;;
    teststd) step pytest_td 600 python -u -m pytest tests/test_gpu_parity.py -k "target_shard" tests/test_gpu_uniform_rows.py tests/test_gpu_log_layout.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab_c2b) step ab_c2b 600 bash -c 'for i in 1 2 3; do for v in default buf3 buf3chk emit1; do echo "== $v"; if [ $v = default ]; then python tools/fuse_probe.py --fuse 16 --repeat 15; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py --fuse 16 --repeat 15; fi; done; done' ;;
    testsrep) step pytest_rep 600 python -u -m pytest tests/test_gpu_replay_fused.py tests/test_gpu_parity.py -k "replay or target_shard or capped" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab_pre) step ab_pre 600 bash -c 'for i in 1 2 3; do for v in default nopre; do echo "== $v"; if [ $v = default ]; then python tools/round_probe.py --workload c4 | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload c4 | tail -1; fi; done; done' ;;
    ab_unc) step ab_unc 900 bash -c 'for w in c5 c4 c4p; do for i in 1 2; do for o in 0 1; do echo "== $w pref_uncached=$o"; python tools/round_probe.py --workload $w --option pref_uncached=$o | tail -1; done; done; done' ;;
    ab_c2p) step ab_c2p 600 bash -c 'for i in 1 2 3; do for v in default pipe3 pipe3late; do echo "== $v"; if [ $v = default ]; then python tools/fuse_probe.py --fuse 16 --repeat 15; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py --fuse 16 --repeat 15; fi; done; done' ;;
    testsrepv) step pytest_repv 600 env AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_${V:-pipe3}.so python -u -m pytest tests/test_gpu_replay_fused.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    c2pmc) step c2pmc 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_INSTS_VALU GRBM_GUI_ACTIVE \
            --output-format csv -d $OUT/c2pmc -o c2 -- python3 tools/fuse_probe.py --fuse 16 --repeat 3 ;;
    gm_ptpw) step gm_ptpw_c4p 600 python tools/group_model.py --workload c4p --ranks 4,8 --kinds masked --variant tpw8:tiles_per_wave=8 --variant tpw4:tiles_per_wave=4 --json $OUT/gm_ptpw_c4p.json && \
             step gm_ptpw_c4pb 600 python tools/group_model.py --workload c4pb --ranks 4,8 --kinds masked --variant tpw8:tiles_per_wave=8 --variant tpw4:tiles_per_wave=4 --json $OUT/gm_ptpw_c4pb.json ;;
    c2abl) step c2abl 300 bash -c 'for i in 1 2; do for o in "replay_fast=1" "ablate_emit=1"; do echo "== $o"; python tools/fuse_probe.py --fuse 16 --repeat 15 --option $o; done; done' ;;
    ab_matnt) step ab_matnt 600 bash -c 'for i in 1 2 3; do for v in default matnt; do echo "== $v"; if [ $v = default ]; then python tools/wb_probe.py --runs 1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/wb_probe.py --runs 1; fi; done; done' ;;
    probes) step probes 600 bash -c 'for w in c4 c4 c5 c4p; do echo "== $w"; python tools/round_probe.py --workload $w | tail -17; done' ;;
    benchx2) step bench_a 900 python bench.py && step bench_b 900 python bench.py ;;
    profc4) step profc4 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc4 -o c4 -- \
            python3 bench.py --no-cpu-baseline --no-secondary ;;
    ab_c3tpw) step ab_c3tpw 600 bash -c 'for i in 1 2; do for t in 4 8 16; do echo "== tpw $t"; python tools/round_probe.py --workload c3 --option tiles_per_wave=$t | tail -1; done; done' ;;
    peers) step pytest_peers 900 python -u -m pytest tests/test_gpu_peer_group.py tests/test_gpu_peer_push.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    gm_c4) step gm_c4 900 python tools/group_model.py --workload c4 --variant nomask:peer_mask=0 --variant tpw16:tiles_per_wave=16 --variant nomask_tpw16:peer_mask=0,tiles_per_wave=16 --json $OUT/group_model_c4.json ;;
    gm_c4p) step gm_c4p 900 python tools/group_model.py --workload c4p --variant nomask:peer_mask=0 --json $OUT/group_model_c4p.json ;;
    gm_c4pb) step gm_c4pb 900 python tools/group_model.py --workload c4pb --variant nomask:peer_mask=0 --json $OUT/group_model_c4pb.json ;;
    ab_c2late) step ab_c2late 600 bash -c 'for i in 1 2 3; do for v in default late; do echo "== $v"; if [ $v = default ]; then python tools/fuse_probe.py | head -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_late.so python tools/fuse_probe.py | head -1; fi; done; done' ;;
    gm_ab) step gm_ab 900 python tools/group_model.py --workload c4p --ranks 8 --kinds targets,masked --variant scoped:push_store=0 --variant ablate:push_store=2 --variant direct:push_defer=0 --variant nomask_abl:peer_mask=0,push_store=2 --variant nomask:peer_mask=0 --json $OUT/group_model_c4p_ab.json ;;
    gm_trace) step gm_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gm_trace -o gm -- \
            python3 tools/group_model.py --workload c4p --ranks 8 --kinds masked --json $OUT/gm_trace.json ;;
    gm_tpw) step gm_tpw 900 python tools/group_model.py --workload c4p --ranks 8 --kinds masked --variant nomask:peer_mask=0 --variant tpw8:tiles_per_wave=8 --variant tpw16:tiles_per_wave=16 --variant nomask_tpw8:peer_mask=0,tiles_per_wave=8 --json $OUT/group_model_c4p_tpw.json ;;
    gm_c4m) step gm_c4m 900 python tools/group_model.py --workload c4 --ranks 8 --kinds targets,masked --target-option uni_merge=4 --variant merge4:uni_merge=4 --variant nomask:peer_mask=0 --variant nomask_merge4:peer_mask=0,uni_merge=4 --json $OUT/group_model_c4_merge.json ;;
    ns_probe) step ns_probe 600 bash -c 'for o in "count_changed=0" "count_changed=1"; do python tools/node_shard_probe.py --workload c4p --shards 1,8 --kinds nodes --rounds 6 --option $o; done' ;;
    gm_merge) step gm_merge 900 python tools/group_model.py --workload c4 --kinds targets --target-option uni_merge=4 --json $OUT/group_model_c4_merge4.json ;;
    pmcea_req) step pmcea_req_${WL:-c5} 600 timeout -s KILL 500 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
            --output-format csv -d $OUT/pmcea_req_${WL:-c5} -o bench -- python3 bench.py --workload ${WL:-c5} --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmcea_dram) step pmcea_dram_${WL:-c5} 600 timeout -s KILL 500 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE \
            --output-format csv -d $OUT/pmcea_dram_${WL:-c5} -o bench -- python3 bench.py --workload ${WL:-c5} --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmcea_sum) step pmcea_sum_${WL:-c5} 120 python tools/pmc_ea.py --req $OUT/pmcea_req_${WL:-c5} --dram $OUT/pmcea_dram_${WL:-c5} --out $OUT/pmc_ea_${WL:-c5}.json ;;
    pmclist) step pmclist 120 rocprofv3 -L ;;
    testsall) step pytest_gpu 1500 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) step bench 900 python bench.py ;;
    rccl2) step rccl2 240 python tools/rccl_two_rank_probe.py ;;
    rehearse2) step rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --rehearse-one-gpu --no-secondary ;;
    rehearse4) step rehearse4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --rehearse-one-gpu --no-secondary ;;
    rehearse2p) step rehearse2p 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --no-secondary --shard peers ;;
    rehearse2s) step rehearse2s 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --rehearse-one-gpu --shard peers ;;
    rehearse8p) step rehearse8p 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --rehearse-one-gpu --no-secondary --workload c4p ;;
    rehearse8) step rehearse8 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 8 --rehearse-one-gpu --no-secondary ;;
    rehearse8all) step rehearse8all 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29540 bench.py --gpus 8 --rehearse-one-gpu ;;
    rehearse4p) step rehearse4p 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --rehearse-one-gpu --no-secondary --shard peers ;;
    capped) step capped 600 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "capped or c2 or replay or fuzz or poll_sets" ;;
    fresh) step fresh 600 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_count_lazy.py tests/test_gpu_virtual_votes.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    probe_c4) step probe_c4 300 python tools/round_probe.py --workload c4 --json $OUT/probe_c4.json ;;
    probe_emit) step probe_emit 300 python tools/round_probe.py --workload c4 --option ablate_emit=1 --json $OUT/probe_c4_noemit.json ;;
    probe_noatomic) step probe_noatomic 300 python tools/round_probe.py --workload c4 --option ablate_emit=2 --json $OUT/probe_c4_noatomic.json ;;
    delivery) step delivery 600 python tools/delivery_probe.py --json $OUT/delivery_c4.json ;;
    probe_c3) step probe_c3 300 python tools/round_probe.py --workload c3 --json $OUT/probe_c3.json ;;
    sq_c4a) step sq_c4a 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq_c4a -o probe -- \
            python3 tools/round_probe.py --workload c4 --warm-epochs 0 ;;
    sq_c4a_noemit) step sq_c4a_noemit 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq_c4a_noemit -o probe -- \
            python3 tools/round_probe.py --workload c4 --warm-epochs 0 --option ablate_emit=1 ;;
    sq_c4b_noemit) step sq_c4b_noemit 300 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_c4b_noemit -o probe -- \
            python3 tools/round_probe.py --workload c4 --warm-epochs 0 --option ablate_emit=1 ;;
    sq_c4b) step sq_c4b 300 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_c4b -o probe -- \
            python3 tools/round_probe.py --workload c4 --warm-epochs 0 ;;
    probe_grid) step probe_grid 600 bash -c 'for o in "sweep_blocks=0" "sweep_blocks=-2" "sweep_blocks=62500" "sweep_blocks=31250" "sweep_blocks=62500 --option sweep_nopipe=1" "sweep_blocks=31250 --option sweep_nopipe=1" "sweep_blocks=7168 --option sweep_nopipe=1"; do echo "== $o"; python tools/round_probe.py --workload c4 --option $o | tail -1; done' ;;
    probe_c3grid) step probe_c3grid 600 bash -c 'for o in "tiles_per_wave=1" "tiles_per_wave=2" "tiles_per_wave=4" "tiles_per_wave=8" "sweep_blocks=0"; do echo "== $o"; python tools/round_probe.py --workload c3 --option $o | tail -1; done' ;;
    probe_runs) step probe_runs 600 bash -c 'for w in c4 c3 c5; do for o in "wave_runs=0" "wave_runs=1"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    probe_fast) step probe_fast 600 bash -c 'for w in c4 c3 c5; do for o in "settled_fast=0" "settled_fast=1"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    newtests) step newtests 900 python -u -m pytest tests/test_gpu_example.py tests/test_gpu_dropin_fuzz.py tests/test_gpu_parity.py tests/test_gpu_delivery.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    dropin) step dropin 300 python tools/dropin_latency.py --json $OUT/dropin_latency.json ;;
    cpptests) step cpptests 300 go-avalanche_amd/bin/avalanche_gpu_tests ;;
    probe_dense) step probe_dense 600 bash -c 'for o in "dense_min=6" "dense_min=4" "dense_min=3" "dense_min=2" "dense_min=1"; do echo "== $o"; python tools/round_probe.py --workload c4 --option $o | head -5; done' ;;
    peertests) step peertests 600 python -u -m pytest tests/test_gpu_peer_push.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    nsprobe) step nsprobe 600 python tools/node_shard_probe.py --json $OUT/node_shard_probe.json ;;
    ab) step ab 900 python tools/ab_tune.py --json $OUT/ab.json ;;
    ab1) step ab1 600 python tools/ab_tune.py --shards 1 --json $OUT/ab1.json ;;
    abc3) step abc3 600 python tools/ab_tune.py --workload c3 --shards 1 --variants sweep,per_tile,ablate --json $OUT/abc3.json ;;
    abpol) step abpol 600 python tools/ab_tune.py --shards 1,8 --variants sweep_w1,sweep_res,w1_sc1,w1_ntsc1,res_sc1,w1_plain --json $OUT/abpol.json ;;
    abres) step abres 600 python tools/ab_tune.py --shards 1,2,4,8 --variants sweep,sweep_w1,sweep_res,ablate --json $OUT/abres.json ;;
    abvv) step abvv 600 python tools/ab_tune.py --shards 1,2,4,8 --variants vv0,sweep,vv_all --json $OUT/abvv.json ;;
    gprobe) step gprobe 120 go-avalanche_amd/bin/gather_probe 20 ;;
    mprobe) step mprobe 120 go-avalanche_amd/bin/mix_probe ;;
    conv_c3) step conv_c3 900 python tools/run_to_finalization.py --workload c3 --json $OUT/conv_c3.json ;;
    conv_c5) step conv_c5 900 python tools/run_to_finalization.py --workload c5 --max-rounds 64 --json $OUT/conv_c5.json ;;
    conv_c4) step conv_c4 900 python tools/run_to_finalization.py --workload c4 --max-rounds 64 --json $OUT/conv_c4.json ;;
    bench_c2) step bench_c2 900 python bench.py --workload c2 --no-cpu-baseline ;;
    bench_c2v1) step bench_c2v1 900 python bench.py --workload c2 --no-cpu-baseline --kernel 1 ;;
    bench_c3) step bench_c3 900 python bench.py --workload c3 --no-cpu-baseline ;;
    bench_c5) step bench_c5 900 python bench.py --workload c5 --no-cpu-baseline ;;
    prof) step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
            python3 bench.py --no-cpu-baseline ;;
    pmcb_sq) step pmcb_sq_${WL:-c4} 600 timeout -s KILL 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
            --output-format csv -d $OUT/pmcb_sq_${WL:-c4} -o bench -- python3 bench.py --workload ${WL:-c4} --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmcb_fetch) step pmcb_fetch_${WL:-c4} 600 timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcb_fetch_${WL:-c4} -o bench -- \
            python3 bench.py --workload ${WL:-c4} --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmcb_write) step pmcb_write_${WL:-c4} 600 timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcb_write_${WL:-c4} -o bench -- \
            python3 bench.py --workload ${WL:-c4} --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmcb_sum) step pmcb_sum_${WL:-c4} 300 python tools/pmc_bench.py --workload ${WL:-c4} --sq $OUT/pmcb_sq_${WL:-c4} --fetch $OUT/pmcb_fetch_${WL:-c4} \
            --write $OUT/pmcb_write_${WL:-c4} --calib-fetch $OUT/calib_fetch --calib-write $OUT/calib_write ${PMC_LAUNCHES:+--launches $PMC_LAUNCHES} ${PMC_REPLAY:+--replay} --out $OUT/pmc_${WL:-c4}.json ;;
    pmc_fetch) step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o bench -- \
            python3 bench.py --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    pmc_write) step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o bench -- \
            python3 bench.py --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    calib_fetch) step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o calib -- \
            go-avalanche_amd/bin/pmc_calib ;;
    calib_write) step calib_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o calib -- \
            go-avalanche_amd/bin/pmc_calib ;;
    pmc_sum) step pmc_sum 120 python tools/pmc_summary.py --calib-fetch $OUT/calib_fetch --calib-write $OUT/calib_write \
            --fetch $OUT/pmc_fetch --write $OUT/pmc_write --kernel k_round_sweep --read-x4 14 --read-x1 64 --write-x4 14 --write-x1 6 --out $OUT/pmc_traffic_c4.json ;;
    pmc_sq8) step pmc_sq8 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq8 -o ab -- \
            python3 tools/ab_tune.py --shards 8 --variants sweep_w1,ablate --rounds 3 ;;
    pmc_tcc8) step pmc_tcc8 300 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_tcc8 -o ab -- \
            python3 tools/ab_tune.py --shards 8 --variants sweep_w1,ablate --rounds 3 ;;
    pmc_sq1) step pmc_sq1 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq1 -o ab -- \
            python3 tools/ab_tune.py --shards 1 --variants sweep_w1 --rounds 3 ;;
    pmc_conv_sq) step pmc_conv_sq 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_conv_sq -o conv -- \
            python3 tools/run_to_finalization.py --workload c4 --max-rounds 20 ;;
    pmc_conv_wr) step pmc_conv_wr 300 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_conv_wr -o conv -- \
            python3 tools/run_to_finalization.py --workload c4 --max-rounds 20 ;;
    pmc_conv_rd) step pmc_conv_rd 300 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_conv_rd -o conv -- \
            python3 tools/run_to_finalization.py --workload c4 --max-rounds 20 ;;
    gaps) step gaps 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps -o gap -- python3 tools/gap_probe.py --workload c4 ;;
    gaps_vv0) step gaps_vv0 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps_vv0 -o gap -- python3 tools/gap_probe.py --workload c4 --option virtual_votes=0 ;;
    gaps40) step gaps40 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps40 -o gap -- python3 tools/gap_probe.py --workload c4 --rounds 40 ;;
    gaps_mk) step gaps_mk 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps_mk -o gap -- python3 tools/gap_probe.py --workload c4 --option round_marker=1 ;;
    gaps_ef) step gaps_ef 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps_ef -o gap -- python3 tools/gap_probe.py --workload c4 --events-first ;;
    gaps2) step gaps2 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps2 -o gap -- python3 tools/gap_probe.py --workload c2 ;;
    profc2) step profc2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc2 -o c2 -- \
            python3 bench.py --workload c2 --no-cpu-baseline ;;
    probe_c2abl) step probe_c2abl 600 bash -c 'for o in "replay_prefetch=0" "replay_prefetch=1" "ablate_node=1" "ablate_node=2" "ablate_node=4" "ablate_emit=1" "ablate_emit=1 --option ablate_node=7"; do echo "== $o"; python tools/round_probe.py --workload c2 --option $o | tail -2; done' ;;
    profc2p) step profc2p 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc2p -o c2 -- \
            python3 tools/round_probe.py --workload c2 ;;
    fused) step fused 600 python -u -m pytest tests/test_gpu_replay_fused.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    fuseprobe) step fuseprobe 300 bash -c 'for o in "ablate_emit=0" "ablate_emit=1" "ablate_emit=2"; do python tools/fuse_probe.py --option $o; done' ;;
    probe_c3opt) step probe_c3opt 600 bash -c 'for o in "virtual_votes=1" "virtual_votes=0" "count_lazy=0" "tiles_per_wave=2" "tiles_per_wave=8" "plane_nt=0" "store_policy=2"; do echo "== $o"; python tools/round_probe.py --workload c3 --option $o | tail -1; done' ;;
    refrows) step refrows 600 python -u -m pytest tests/test_gpu_ref_rows.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    probe_ref) step probe_ref 300 bash -c 'for o in "ref_rows=1" "ref_rows=0"; do echo "== $o"; python tools/round_probe.py --workload c4 --option $o; done' ;;
    nstpw) step nstpw 600 bash -c 'for o in "tiles_per_wave=4" "tiles_per_wave=2" "tiles_per_wave=1"; do python tools/node_shard_probe.py --shards 1,2,4,8 --kinds nodes --option $o; done' ;;
    probe_settled) step probe_settled 600 bash -c 'for o in "ablate_settled=0" "ablate_settled=1" "ablate_settled=2" "ablate_settled=4" "ablate_settled=8" "ablate_settled=15" "ablate_settled=7"; do echo "== $o"; python tools/round_probe.py --workload c4 --option $o | grep "\"round\": 1[0-2],"; done' ;;
    benchwin) step benchwin 900 bash -c 'python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary && python bench.py --steps 5 --warmup 0 --no-cpu-baseline --no-secondary && python bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-secondary' ;;
    probe_tpw) step probe_tpw 600 bash -c 'for w in c4 c3; do for o in "tiles_per_wave=4" "tiles_per_wave=6" "tiles_per_wave=8" "tiles_per_wave=3"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o | tail -1 | grep -o "kernel_ms_total.*"; done; done' ;;
    c4ptests) step c4ptests 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -k "c4p" ;;
    hostcpu) step hostcpu 300 bash -c 'cat /sys/fs/cgroup/cpu.max; nproc; python -c "import bench, json; print(json.dumps(bench.host_cpus()))"; for t in 16 32 64 128; do python tools/cpu_scaling.py --threads $t; done' ;;
    bench_c4p) step bench_c4p 900 python bench.py --workload c4p --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    bench_c4pb) step bench_c4pb 900 python bench.py --workload c4pb --no-cpu-baseline --no-secondary --no-exchange-pass ;;
    probe_lean) step probe_lean 600 bash -c 'for w in c4 c5; do for o in "settled_lean=1" "settled_lean=0"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    fullc4) step fullc4 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -k "c4_fullsize" ;;
    probe_ref2) step probe_ref2 600 bash -c 'for w in c4 c5; do for o in "ref_rows=1" "ref_rows=0"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    reftests) step reftests 900 python -u -m pytest tests/test_gpu_ref_rows.py tests/test_gpu_virtual_votes.py tests/test_gpu_fresh.py tests/test_gpu_count_lazy.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    fullc5) step fullc5 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -k "c5" ;;
    dropintests) step dropintests 600 python -u -m pytest tests/test_gpu_dropin_fuzz.py tests/test_gpu_example.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abuni) step abuni 600 bash -c 'for w in c4 c5 c4p; do for o in uniform_rows=1 uniform_rows=0; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    unitests) step unitests 900 python -u -m pytest tests/test_gpu_uniform_rows.py tests/test_gpu_count_lazy.py tests/test_gpu_ref_rows.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abtpw) step abtpw 600 bash -c 'for w in c4 c4p; do for o in tiles_per_wave=16 tiles_per_wave=8; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    abub) step abub 600 bash -c 'for w in c4 c5 c3; do for o in uni_blocks=-1 uni_blocks=2560 uni_blocks=5120 uni_blocks=0; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    abhv) step abhv 600 bash -c 'for w in c4 c4pb c3; do for o in k_hi_virtual=1 k_hi_virtual=0; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    hvtests) step hvtests 900 python -u -m pytest tests/test_gpu_count_lazy.py tests/test_gpu_fresh.py tests/test_gpu_virtual_votes.py tests/test_gpu_uniform_rows.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    barrier) step barrier 300 bash -c 'python tools/barrier_cost.py --world 2 --json gpurun_out/barrier2.json && python tools/barrier_cost.py --world 4 --json gpurun_out/barrier4.json && python tools/barrier_cost.py --world 2 --nodes 131072 --json gpurun_out/barrier2_big.json' ;;
    evidence) for S in abtpw abuni abhv; do bash "$0" $S || exit $?; done ;;
    abmerge) step abmerge 600 bash -c 'for w in c4 c5 c4p; do for o in uni_merge=2 uni_merge=1 uni_merge=4; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o; done; done' ;;
    barrierfine) step barrierfine 300 bash -c 'python tools/barrier_cost.py --world 2 --nodes 131072 --option peer_fine=0 --json gpurun_out/barrier2_big_coarse.json && python tools/barrier_cost.py --world 2 --nodes 131072 --json gpurun_out/barrier2_big_fine.json && python tools/barrier_cost.py --world 2 --nodes 1000000 --option peer_fine=0 --rounds 40 --json gpurun_out/barrier2_c4_coarse.json && python tools/barrier_cost.py --world 2 --nodes 1000000 --rounds 40 --json gpurun_out/barrier2_c4_fine.json' ;;
    barrierfold) step barrierfold 300 bash -c 'for o in fold_arrival=0 fold_arrival=1; do python tools/barrier_cost.py --world 2 --nodes 131072 --option $o --json gpurun_out/barrier2_big_$o.json && python tools/barrier_cost.py --world 2 --nodes 1000000 --rounds 40 --option $o --json gpurun_out/barrier2_c4_$o.json && python tools/barrier_cost.py --world 2 --option $o --json gpurun_out/barrier2_small_$o.json || exit 1; done' ;;
    abw6) step abw6 600 bash -c 'for w in c4 c4p c4pb; do for v in base w6 w7; do echo "== $w $v"; if [ $v = base ]; then python tools/round_probe.py --workload $w; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w; fi; done; done' ;;
    mall) step mall 600 python tools/mall_probe.py --workload c4p --shards 1,8 --kinds nodes,targets --json $OUT/mall_probe_c4p.json ;;
    gm_warm) step gm_warm_c4p 900 python tools/group_model.py --workload c4p --ranks 8 --kinds targets,masked --all-option warm_pref=1 --json $OUT/gm_warm_c4p.json && \
             step gm_cold_c4p 900 python tools/group_model.py --workload c4p --ranks 8 --kinds targets,masked --json $OUT/gm_cold_c4p.json && \
             step gm_warm_c4 900 python tools/group_model.py --workload c4 --ranks 8 --kinds targets,masked --all-option warm_pref=1 --json $OUT/gm_warm_c4.json ;;
    smaxtests) step smaxtests 900 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_delivery.py tests/test_gpu_log_layout.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab_smax) step ab_smax 900 bash -c 'for i in 1 2; do for w in c4p c4 c4pb; do for v in default smax1; do echo "== $w $v"; if [ $v = default ]; then python tools/round_probe.py --workload $w --rounds 8 | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w --rounds 8 | tail -1; fi; done; done; done' ;;
    ab_wd) step ab_wd 900 bash -c 'for i in 1 2; do for w in c4p c4; do for o in "wave_dense=0" "wave_dense=32" "wave_dense=1"; do echo "== $w $o"; python tools/round_probe.py --workload $w --rounds 6 --option $o | tail -7; done; done; done' ;;
    wdtests) step wdtests 600 env AVHIP_TEST_OPTIONS=wave_dense=1 python -u -m pytest tests/test_gpu_compact.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab_uv) step ab_uv 900 bash -c 'for i in 1 2; do for w in c4 c5; do for o in "uni_votes=1" "uni_votes=0"; do echo "== $w $o"; python tools/round_probe.py --workload $w --rounds 10 --option $o | tail -11; done; done; done' ;;
    uvtests) step uvtests 900 python -u -m pytest tests/test_gpu_uniform_rows.py tests/test_gpu_bench_protocol.py tests/test_gpu_count_lazy.py tests/test_gpu_virtual_votes.py tests/test_gpu_fullsize.py -k "uniform or uni_ or protocol or lazy or virtual or c4_fullsize or c5_whole" -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    pmcall) for W in c4 c4p c4pb c3 c5; do WL=$W bash "$0" pmcb_sq pmcb_fetch pmcb_write pmcb_sum || exit $?; done
            WL=c2 PMC_LAUNCHES=2 PMC_REPLAY=1 bash "$0" pmcb_sq pmcb_fetch pmcb_write pmcb_sum || exit $? ;;
    bench4) step bench 900 python bench.py --detail gpurun_out/bench_detail.json ;;
    self2) step self2 600 python bench.py --gpus 2 --rehearse-one-gpu --no-secondary --detail gpurun_out/rehearse2_detail.json ;;
    self2s) step self2s 900 python bench.py --gpus 2 --rehearse-one-gpu --detail gpurun_out/rehearse2s_detail.json ;;
    exchcost) step exchcost 300 python tools/exchange_cost.py --json gpurun_out/exchange_cost.json ;;
    barrier4) step barrier4 400 bash -c 'python tools/barrier_cost.py --world 2 --json gpurun_out/barrier2_small.json && python tools/barrier_cost.py --world 2 --nodes 131072 --json gpurun_out/barrier2_big.json && python tools/barrier_cost.py --world 4 --nodes 131072 --json gpurun_out/barrier4_big.json && python tools/barrier_cost.py --world 2 --nodes 1000000 --rounds 40 --json gpurun_out/barrier2_c4.json' ;;
    abr3) step abr3 600 bash -c 'for w in c4 c4p c4pb; do for v in new nohoist r3; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done; for v in new r3; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    ablate) step ablate 600 bash -c 'for w in c4 c4p; do for o in "ablate_phase=0" "ablate_phase=1" "ablate_phase=2" "ablate_phase=4" "ablate_phase=16" "ablate_emit=1" "ablate_phase=7 --option ablate_emit=1"; do echo "== $w $o"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_ablate.so python tools/round_probe.py --workload $w --rounds 8 --option $o | grep -v "^{\"workload"; done; done' ;;
    quick) step quick 900 python -u -m pytest tests/test_gpu_peer_push.py tests/test_gpu_parity.py tests/test_gpu_uniform_rows.py tests/test_gpu_count_lazy.py tests/test_gpu_virtual_votes.py tests/test_gpu_fresh.py tests/test_gpu_replay_fused.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    tshard) step tshard 600 bash -c 'for o in tiles_per_wave=4 tiles_per_wave=8 tiles_per_wave=16; do python tools/shard_model.py --workload c4 --kinds targets --no-one-gpu --ranks 2,4,8 --option $o --json gpurun_out/tshard_c4_$o.json | tail -3; done' ;;
    shardmodel2) step shardmodel2 600 bash -c 'python tools/shard_model.py --workload c4 --json gpurun_out/shard_model_c4.json && python tools/shard_model.py --workload c4p --json gpurun_out/shard_model_c4p.json && python tools/shard_model.py --workload c4pb --json gpurun_out/shard_model_c4pb.json' ;;
    abuni4) step abuni4 600 bash -c 'for w in c4 c5 c4pb; do for v in new s3; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w; fi; done; done' ;;
    abdense) step abdense 600 bash -c 'for w in c4 c4p c4pb; do for v in new dense2 dense4; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done' ;;
    abs4) step abs4 900 bash -c 'for w in c4 c4p c4pb; do for v in new walk walk0; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w; fi; done; done; for v in new walk0; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    tsparity) step tsparity 600 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "target_shard" ;;
    abemit) step abemit 600 bash -c 'for w in c4p c4; do for o in 0 1 2 3; do echo "== $w ablate_emit=$o"; python tools/round_probe.py --workload $w --option ablate_emit=$o | tail -1; done; done' ;;
    ablate5) step ablate5 600 bash -c 'for w in c4p; do for o in "ablate_phase=0" "ablate_phase=1" "ablate_phase=2" "ablate_phase=4" "ablate_phase=16" "ablate_emit=1" "ablate_phase=7 --option ablate_emit=1"; do echo "== $w $o"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_ablate.so python tools/round_probe.py --workload $w --rounds 8 --option $o | grep -v "^{\"workload"; done; done' ;;
    tshard2) step tshard2 600 python tools/shard_model.py --workload c4 --kinds targets --ranks 2,4,8 --json gpurun_out/tshard_c4_default.json ;;
    c2x) step c2x 600 bash -c 'AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_c2x.so python -u -m pytest tests/test_gpu_replay_fused.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "replay or c2 or capped or fused" && for v in new c2x new c2x; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    full4p) step full4p 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bench_protocol.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    abs5) step abs5 900 bash -c 'for w in c4 c4p c4pb; do for v in new walk0; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w; fi; done; done; for v in new walk0 new walk0; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    abpad) step abpad 900 bash -c 'for w in c4p c4 c4pb c4p; do for v in new pad; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done; for o in 2 3; do echo "== c4p pad ablate_emit=$o"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_pad.so python tools/round_probe.py --workload c4p --option ablate_emit=$o | tail -1; done; for v in new pad; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    quicktwo) step quicktwo 900 env AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_two.so python -u -m pytest tests/test_gpu_peer_push.py tests/test_gpu_parity.py tests/test_gpu_uniform_rows.py tests/test_gpu_count_lazy.py tests/test_gpu_virtual_votes.py tests/test_gpu_fresh.py tests/test_gpu_replay_fused.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abtwo) step abtwo 900 bash -c 'for w in c4p c4pb c4 c4p; do for v in pad two; do echo "== $w $v"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; done; done; for v in pad two; do echo "== c2 $v"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; done' ;;
    profc4) step profc4 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc4 -o c4 -- python3 bench.py --no-cpu-baseline --no-secondary ;;
    ablognt) step ablognt 600 bash -c 'for w in c4p c4 c4pb c4p; do for v in new lognt; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done' ;;
    abpub) step abpub 600 bash -c 'for w in c4p c4 c4pb c4p; do for v in new pubplain sp3; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; elif [ $v = sp3 ]; then python tools/round_probe.py --workload $w --option store_policy=3 | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done' ;;
    abwpe) step abwpe 600 bash -c 'for w in c4p c4 c4pb c4p c4; do for v in new w5 w7; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done' ;;
    abwpe2) step abwpe2 600 bash -c 'for w in c4p c4 c4pb c4p c4 c5 c3; do for v in new w5 w4; do echo "== $w $v"; if [ $v = new ]; then python tools/round_probe.py --workload $w | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w | tail -1; fi; done; done' ;;
    abf5) step abf5 600 bash -c 'for w in c4 c4p c4 c4p c4pb c5; do for v in w5 f5; do echo "== $w $v"; AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w > gpurun_out/rp_tmp.txt 2>/dev/null; head -1 gpurun_out/rp_tmp.txt; tail -1 gpurun_out/rp_tmp.txt; done; done' ;;
    self4s) step self4s 900 python bench.py --gpus 4 --rehearse-one-gpu --detail gpurun_out/rehearse4s_detail.json ;;
    abrun8) step abrun8 600 bash -c 'for w in c4 c4p c4 c4p c4pb; do for o in "tiles_per_wave=0 --option uni_merge=1" "tiles_per_wave=8 --option uni_merge=2" "tiles_per_wave=4 --option uni_merge=4"; do echo "== $w $o"; python tools/round_probe.py --workload $w --option $o | tail -1; done; done' ;;
    abc5tpw) step abc5tpw 600 bash -c 'for w in c5 c5; do for o in 0 4 16; do echo "== $w tpw=$o"; python tools/round_probe.py --workload $w --option tiles_per_wave=$o | tail -1; done; done' ;;
    c2ab) step c2ab 300 bash -c 'for v in new s3; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    reh2pb) step reh2pb 600 python bench.py --gpus 2 --rehearse-one-gpu --workload c4pb --shard peers --no-secondary --detail gpurun_out/rehearse2_c4pb_detail.json ;;
    reh2t) step reh2t 600 python bench.py --gpus 2 --rehearse-one-gpu --shard targets --no-secondary --detail gpurun_out/rehearse2_targets_detail.json ;;
    abs3) step abs3 900 bash -c 'for w in c4 c4p c4pb c3; do for v in new s3; do for cc in 0 1; do echo "== $w $v count_changed=$cc"; if [ $v = new ]; then python tools/round_probe.py --workload $w --option count_changed=$cc | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w --option count_changed=$cc | tail -1; fi; done; done; done; for v in new s3; do echo "== c2 $v"; if [ $v = new ]; then python tools/fuse_probe.py; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/fuse_probe.py; fi; done' ;;
    profc2b) step profc2b 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc2b -o c2 -- python3 bench.py --workload c2 --no-cpu-baseline --no-secondary ;;
    abcc) step abcc 600 bash -c 'for w in c4 c4p; do for v in new noccpf; do for cc in 0 1; do echo "== $w $v count_changed=$cc"; if [ $v = new ]; then python tools/round_probe.py --workload $w --option count_changed=$cc | tail -1; else AVHIP_LIB=go-avalanche_amd/lib/variants/libavhip_$v.so python tools/round_probe.py --workload $w --option count_changed=$cc | tail -1; fi; done; done; done; python tools/round_probe.py --workload c4pb | tail -1' ;;
    shardmodel) step shardmodel 600 bash -c 'python tools/shard_model.py --workload c4 --json gpurun_out/shard_model_c4.json && python tools/shard_model.py --workload c4p --json gpurun_out/shard_model_c4p.json' ;;
    fused4) step fused4 600 python -u -m pytest tests/test_gpu_replay_fused.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    peer4) step peer4 600 python -u -m pytest tests/test_gpu_peer_push.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session done" | tee -a $OUT/session.log
