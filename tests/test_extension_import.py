"""The built extension registers its operator schemas without a GPU (CPU check).

A bad ``TORCH_LIBRARY`` schema aborts the process at import time, so the import runs in
a child process; skipped when the extension has not been built in-tree.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_extension_imports_and_registers_ops():
    if not any(f.startswith('_C') and f.endswith('.so')
               for f in os.listdir(os.path.join(ROOT, 'torchgpipe_amd'))):
        pytest.skip('extension not built (python -m torchgpipe_amd._build)')
    code = ('import torch, torchgpipe_amd._C; '
            'ops = torch.ops.tgpipe; '
            'names = ["convbn_forward", "convbn_backward", "conv_gemm_backward_weight", '
            '"avgpool3_forward", "bn_train_forward"]; '
            'print(all(hasattr(ops, n) for n in names))')
    out = subprocess.run([sys.executable, '-c', code], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().endswith('True')


def test_shipped_plan_table_loads():
    """The shipped MI355X plan table parses and every entry is a valid launch shape."""
    table = os.path.join(ROOT, 'torchgpipe_amd', 'tuned', 'conv_gemm_mi355x.txt')
    if not os.path.exists(table) or not any(
            f.startswith('_C') and f.endswith('.so')
            for f in os.listdir(os.path.join(ROOT, 'torchgpipe_amd'))):
        pytest.skip('extension or plan table missing')
    with open(table) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip()]
    code = ('import os; os.environ["TGPIPE_CG_DB"] = "0"; import torch, torchgpipe_amd._C; '
            'from torchgpipe_amd.ops import _ext; '
            f'print(_ext.load_plans({table!r}), '
            'torch.ops.tgpipe.conv_gemm_plans_export().count(chr(10)))')
    out = subprocess.run([sys.executable, '-c', code], cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    taken, exported = map(int, out.stdout.split()[-2:])
    assert taken == len(lines) == exported
