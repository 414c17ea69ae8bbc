#!/bin/bash
# r5y: host cost of stream / event primitives and of the AmoebaNet / ResNet units
export TMPDIR=/tmp
out=gpurun_out/r5y
mkdir -p $out
timeout -k 10 300 python -u benchmarks/host_cell.py --out $out/host_cell.json > $out/host_cell.log 2>&1 || { tail -20 $out/host_cell.log; exit 1; }
cat $out/host_cell.json
