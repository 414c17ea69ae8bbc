#!/bin/bash
# r5bc: AmoebaNet n1m32 bench (captured cells) under engine options: cell streams 2 / 3,
# weight-gradient stream, recompute lane
export TMPDIR=/tmp
out=gpurun_out/r5bc
mkdir -p $out
b() { name=$1; shift; timeout -k 10 400 env "$@" > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }; python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', d['value'], d['ms_per_step'])"; }

b recompute_lane TGPIPE_X=1 python3 bench.py --gpus 1 --model amoebanet --steps 5 --warmup 3 --sections none --overlap-recompute on
b default2 TGPIPE_X=1 python3 bench.py --gpus 1 --model amoebanet --steps 5 --warmup 3 --sections none
