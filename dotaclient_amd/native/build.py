"""Build the native host-side module ``dotaclient_amd/native/_native*.so`` (C++17, pybind11, no torch):
protobuf wire decoder + featurizer, shared-memory experience ring, crc32c. ``python -m dotaclient_amd.native.build``."""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'featurizer.cpp')
TARGET = os.path.join(HERE, '_native' + (sysconfig.get_config_var('EXT_SUFFIX') or '.so'))


def build(verbose: bool = True, force: bool = False, debug_asan: bool = False) -> str:
    if not force and os.path.exists(TARGET) and os.path.getmtime(TARGET) > os.path.getmtime(SRC) and not debug_asan:
        return TARGET
    import pybind11
    cxx = os.environ.get('CXX', 'g++')
    flags = ['-O3', '-std=c++17', '-fPIC', '-shared', '-msse4.2', '-pthread', '-Wall', '-Wno-unused-function']
    target = TARGET
    if debug_asan:   # host-side sanitizer build (race / memory checks of the ring + decoder)
        flags = ['-O1', '-g', '-std=c++17', '-fPIC', '-shared', '-msse4.2', '-pthread', '-fsanitize=address,undefined',
                 '-fno-omit-frame-pointer']
        target = os.path.join(HERE, '_native_asan' + (sysconfig.get_config_var('EXT_SUFFIX') or '.so'))
    cmd = [cxx, *flags, '-I', pybind11.get_include(), '-I', sysconfig.get_paths()['include'], SRC, '-o', target, '-lrt']
    if verbose:
        print('[dotaclient_amd.native] ' + ' '.join(cmd[:3]) + ' ...', flush=True)
    subprocess.run(cmd, check=True)
    return target


if __name__ == '__main__':
    build(force='--force' in sys.argv, debug_asan='--asan' in sys.argv)
