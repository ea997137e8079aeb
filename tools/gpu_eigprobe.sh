#!/bin/bash
# Eigensolver concurrency probe (tools/probe_eig.cpp, built in-tree as tools/bin/probe_eig).
set -o pipefail
OUT=gpurun_out/r03/eig
mkdir -p $OUT
echo "[$(date +%T)] eig 8192" && \
timeout -k 10 240 tools/bin/probe_eig 8192 8 > $OUT/eig8192.jsonl 2> $OUT/eig.err && cat $OUT/eig8192.jsonl && \
echo "[$(date +%T)] eig 16384" && \
timeout -k 10 400 tools/bin/probe_eig 16384 4 > $OUT/eig16384.jsonl 2>> $OUT/eig.err && cat $OUT/eig16384.jsonl && \
echo "[$(date +%T)] done"
