"""In-tree builder for the gfx950 HIP extension ``dotaclient_amd/ops/_C*.so`` (and the native host libraries).

No hipify, no torch JIT cache: every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an
object file (these TUs include no torch headers, so they rebuild in seconds), ``csrc/bindings.cpp`` is compiled once
against torch's headers, and everything is linked into one shared object next to this file — so it travels with the
repository snapshot to the GPU box and is what the tests load. Rebuilds are incremental (mtime of source vs object,
any header change rebuilds all).

    python -m dotaclient_amd.ops.build          # build (cross-compiles fine on a CPU-only host)
    python -m dotaclient_amd.ops.build --clean
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, '_build')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
EXT_SUFFIX = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
TARGET = os.path.join(HERE, '_C' + EXT_SUFFIX)

COMMON_FLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-D__HIP_PLATFORM_AMD__=1',
                '-Wno-unused-result', '-Wno-unused-command-line-argument']


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = [os.path.join(os.path.dirname(torch.__file__), 'include'),
           os.path.join(os.path.dirname(torch.__file__), 'include', 'torch', 'csrc', 'api', 'include')]
    lib = os.path.join(os.path.dirname(torch.__file__), 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _needs(obj: str, srcs) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError(f'command failed ({p.returncode}): {" ".join(cmd)}\n{p.stdout}')
    return p.stdout


def build(verbose: bool = True, jobs: int = 8, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, '*.h'))
    hips = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()['include']
    objs, jobs_list = [], []
    for src in hips:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        if force or _needs(obj, [src] + headers):
            jobs_list.append([HIPCC, *COMMON_FLAGS, '-I', CSRC, '-c', src, '-o', obj])
    bsrc = os.path.join(CSRC, 'bindings.cpp')
    bobj = os.path.join(BUILD, 'bindings.cpp.o')
    objs.append(bobj)
    if force or _needs(bobj, [bsrc] + headers):
        jobs_list.append([HIPCC, *COMMON_FLAGS, '-I', CSRC, *sum([['-I', i] for i in inc], []), '-I', py_inc,
                          '-DTORCH_EXTENSION_NAME=_C', '-DTORCH_API_INCLUDE_EXTENSION_H', '-DUSE_ROCM=1',
                          f'-D_GLIBCXX_USE_CXX11_ABI={abi}', '-c', bsrc, '-o', bobj])
    if jobs_list:
        if verbose:
            print(f'[dotaclient_amd.ops] compiling {len(jobs_list)} translation unit(s) for {ARCH}', flush=True)
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for f in [ex.submit(_run, c) for c in jobs_list]:
                f.result()
    if force or jobs_list or _needs(TARGET, objs):
        _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', *objs, '-o', TARGET, '-L', lib,
              f'-Wl,-rpath,{lib}', '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip', '-ltorch_python'])
        if verbose:
            print(f'[dotaclient_amd.ops] linked {TARGET}', flush=True)
    return TARGET


def clean():
    shutil.rmtree(BUILD, ignore_errors=True)
    if os.path.exists(TARGET):
        os.remove(TARGET)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--clean', action='store_true')
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', '--jobs', type=int, default=int(os.environ.get('MAX_JOBS', '8')))
    a = ap.parse_args(argv)
    if a.clean:
        clean()
        return
    build(jobs=a.jobs, force=a.force)


if __name__ == '__main__':
    main()
