"""In-tree build of the native extension ``torchgpipe_amd/_C.so`` for gfx950.

No hipify, no CUDA paths: ``kernels.hip`` is plain HIP compiled by ``hipcc
--offload-arch=gfx950``; ``bindings.cpp`` is host-only C++ against the
PyTorch-ROCm headers (``ATen/hip``).  Objects are cached under ``build/``
and rebuilt only when a source or header is newer.

Usage::

    python -m torchgpipe_amd._build          # build (incremental)
    python -m torchgpipe_amd._build --force  # rebuild everything
"""
import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(ROOT, 'build', 'tgpipe')
TARGET = os.path.join(HERE, '_C.so')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')

KERNEL_SOURCES = ['kernels.hip', 'winograd.hip', 'winograd_f4.hip', 'conv_gemm.hip',
                  'batchnorm.hip', 'pool.hip', 'unet_ops.hip']
HOST_SOURCES = ['bindings.cpp', 'convbn.cpp']
HEADERS = ['kernels.h', 'philox.h']


def _torch_dirs() -> List[str]:
    import torch
    base = os.path.dirname(torch.__file__)
    return [os.path.join(base, 'include'),
            os.path.join(base, 'include', 'torch', 'csrc', 'api', 'include')]


def _torch_lib() -> str:
    import torch
    return os.path.join(os.path.dirname(torch.__file__), 'lib')


def _cxx11_abi() -> int:
    import torch
    return int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _stale(obj: str, deps: List[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(' '.join(cmd), flush=True)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError(f'native build failed: {cmd[0]} exited {proc.returncode}')
    elif verbose and proc.stdout.strip():
        print(proc.stdout)


def hipcc() -> str:
    path = os.path.join(ROCM, 'bin', 'hipcc')
    return path if os.path.exists(path) else (shutil.which('hipcc') or 'hipcc')


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile (incrementally) and link ``_C.so``; returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in HEADERS]
    objects: List[str] = []
    relink = force or not os.path.exists(TARGET)

    common = ['-O3', '-fPIC', '-std=c++17', '-D__HIP_PLATFORM_AMD__=1']
    for src in KERNEL_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, src + '.o')
        if force or _stale(obj, [path] + headers):
            _run([hipcc(), f'--offload-arch={ARCH}', *common, '-munsafe-fp-atomics',
                  '-c', path, '-o', obj], verbose)
            relink = True
        objects.append(obj)

    py_inc = sysconfig.get_paths()['include']
    torch_inc = [f'-I{d}' for d in _torch_dirs()]
    for src in HOST_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, src + '.o')
        if force or _stale(obj, [path] + headers):
            _run(['g++', *common, '-DUSE_ROCM=1', '-DTORCH_API_INCLUDE_EXTENSION_H',
                  '-DTORCH_EXTENSION_NAME=_C', f'-D_GLIBCXX_USE_CXX11_ABI={_cxx11_abi()}',
                  f'-I{ROCM}/include', *torch_inc, f'-I{py_inc}', '-c', path, '-o', obj],
                 verbose)
            relink = True
        objects.append(obj)

    if relink:
        lib = _torch_lib()
        _run([hipcc(), f'--offload-arch={ARCH}', '-shared', '-fPIC', *objects, '-o', TARGET,
              f'-L{lib}', '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip',
              '-ltorch_python', f'-Wl,-rpath,{lib}', f'-L{ROCM}/lib', '-lamdhip64'], verbose)
    return TARGET


def main() -> None:
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('--force', action='store_true')
    parser.add_argument('-v', '--verbose', action='store_true')
    args = parser.parse_args()
    print(build(force=args.force, verbose=args.verbose))


if __name__ == '__main__':
    main()
