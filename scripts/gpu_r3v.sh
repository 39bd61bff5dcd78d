#!/bin/bash
# round 3, session 3: host-to-device copies captured into a graph (pageable / pinned source
# rewritten after capture) with packet capture on and off; no kernel here indexes memory
# with data, so a broken node cannot fault
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/probe_graph_nodes.py --rounds 50 > gpurun_out/r3v_nodes_pc_default.log 2>&1 || { tail -20 gpurun_out/r3v_nodes_pc_default.log; exit 1; }
grep nodes gpurun_out/r3v_nodes_pc_default.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u scripts/probe_graph_nodes.py --rounds 50 > gpurun_out/r3v_nodes_pc0.log 2>&1 || { tail -20 gpurun_out/r3v_nodes_pc0.log; exit 1; }
grep nodes gpurun_out/r3v_nodes_pc0.log
