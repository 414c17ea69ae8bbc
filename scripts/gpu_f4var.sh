set -o pipefail
timeout -k 10 300 python benchmarks/wino_variants.py --variants 14 16 15 17 --shape 40 1024 1024 12 --shape 40 512 512 24 --shape 16 512 512 24 --shape 16 2048 2048 6 > gpurun_out/abl.log 2>&1 || { tail gpurun_out/abl.log; exit 1; }
timeout -k 10 300 python -c "
import torch, json, sys
sys.path.insert(0, '.')
from torchgpipe_amd.ops import _ext
ops = _ext.require()
for n, c, k, h in [(40, 1024, 1024, 12), (40, 512, 512, 24), (16, 2048, 2048, 6)]:
    x = torch.randn(n, c, h, h, device='cuda'); dy = torch.randn(n, k, h, h, device='cuda')
    row = {'shape': [n, c, k, h]}
    for v in (1, 2):
        for _ in range(3): ops.wino4_wgrad(x, dy, 0, v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): ops.wino4_wgrad(x, dy, 0, v)
        e.record(); e.synchronize(); row[f'wg{v}'] = round(s.elapsed_time(e) / 20, 4)
    print(json.dumps(row))
" > gpurun_out/wgabl.log 2>&1 || { tail gpurun_out/wgabl.log; exit 1; }
echo DONE
