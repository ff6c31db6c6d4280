"""Build the native host-side module ``dotaclient_amd/native/_native*.so`` (C++17, pybind11, no torch):
protobuf wire decoder + featurizer, shared-memory experience ring, crc32c. ``python -m dotaclient_amd.native.build``.

``build_sanitizer('asan' | 'tsan')`` builds the standalone sanitizer driver (``sanitize_main.cpp`` over ``core.h``)
under AddressSanitizer + UndefinedBehaviorSanitizer or ThreadSanitizer (host code only)."""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'featurizer.cpp')
CORE = os.path.join(HERE, 'core.h')
VECENV = os.path.join(HERE, 'vecenv.h')
TARGET = os.path.join(HERE, '_native' + (sysconfig.get_config_var('EXT_SUFFIX') or '.so'))


def build(verbose: bool = True, force: bool = False) -> str:
    if (not force and os.path.exists(TARGET)
            and os.path.getmtime(TARGET) > max(os.path.getmtime(p) for p in (SRC, CORE, VECENV))):
        return TARGET
    import pybind11
    cxx = os.environ.get('CXX', 'g++')
    # -ffp-contract=off: no FMA contraction — the vectorised engine reproduces the python oracle bit for bit
    flags = ['-O3', '-std=c++17', '-fPIC', '-shared', '-msse4.2', '-pthread', '-Wall', '-Wno-unused-function',
             '-ffp-contract=off']
    target = TARGET
    cmd = [cxx, *flags, '-I', pybind11.get_include(), '-I', sysconfig.get_paths()['include'], SRC, '-o', target, '-lrt']
    if verbose:
        print('[dotaclient_amd.native] ' + ' '.join(cmd[:3]) + ' ...', flush=True)
    subprocess.run(cmd, check=True)
    return target


SANITIZE_FLAGS = {
    'asan': ['-fsanitize=address,undefined', '-fno-sanitize-recover=undefined', '-fno-omit-frame-pointer'],
    'tsan': ['-fsanitize=thread'],
}


def build_sanitizer(kind: str = 'asan', verbose: bool = False) -> str:
    """Compile the sanitizer driver for ``kind`` into ``native/_build/sanitize_<kind>``; returns its path."""
    out_dir = os.path.join(HERE, '_build')
    os.makedirs(out_dir, exist_ok=True)
    target = os.path.join(out_dir, f'sanitize_{kind}')
    src = os.path.join(HERE, 'sanitize_main.cpp')
    if os.path.exists(target) and os.path.getmtime(target) > max(os.path.getmtime(src), os.path.getmtime(CORE)):
        return target
    cxx = os.environ.get('CXX', 'g++')
    cmd = [cxx, '-O1', '-g', '-std=c++17', '-msse4.2', '-pthread', *SANITIZE_FLAGS[kind], src, '-o', target, '-lrt']
    if verbose:
        print('[dotaclient_amd.native] ' + ' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return target


if __name__ == '__main__':
    if '--sanitize' in sys.argv:
        for k in ('asan', 'tsan'):
            print(build_sanitizer(k, verbose=True))
    else:
        build(force='--force' in sys.argv)
