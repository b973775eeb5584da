#!/usr/bin/env python3
"""Build every native component in-tree (no JIT cache, no pip install).

* ``kiosk_autoscaler_amd/ops/_kiosk_hip<ext>`` -- gfx950 kernels
  (csrc/kernels/*.hip) + runtime (csrc/runtime/*.cpp: engine, RCCL fence,
  pybind11 bindings), compiled with ``hipcc --offload-arch=gfx950`` and
  linked ``-shared -fPIC``.  RCCL is dlopen'ed at run time (see fence.hpp).
* ``build/kredis-server`` -- the native RESP server (csrc/kredis), g++.
* ``--fake-hip``: ``build/fake/_kiosk_fence_cpu<ext>`` -- the node
  communicator bindings (RCCL Fence + ShmComm, csrc/runtime/bind_comm.cpp)
  built with g++ for the CPU against ``build/fake/libkiosk_fake_hip_rccl.so``
  (csrc/fakes: shared-memory multi-process HIP + RCCL stand-ins), so the
  production fence code runs in N CPU processes (``KIOSK_NATIVE=fake``).

Objects are cached by source mtime under ``build/obj``; ``--clean`` rebuilds.
"""
import argparse
import concurrent.futures
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, 'build')
OBJ = os.path.join(BUILD, 'obj')
ARCH = os.environ.get('KIOSK_OFFLOAD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
EXT = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
EXT_PATH = os.path.join(ROOT, 'kiosk_autoscaler_amd', 'ops', '_kiosk_hip' + EXT)
KREDIS = os.path.join(BUILD, 'kredis-server')
RCCL_SLIM = os.path.join(BUILD, 'kiosk-rccl-slim')
FAKE_DIR = os.path.join(BUILD, 'fake')
FAKE_LIB = os.path.join(FAKE_DIR, 'libkiosk_fake_hip_rccl.so')
FAKE_EXT = os.path.join(FAKE_DIR, '_kiosk_fence_cpu' + EXT)


def _includes():
    import pybind11
    return ['-I' + pybind11.get_include(),
            '-I' + sysconfig.get_paths()['include'],
            '-I' + os.path.join(ROOT, 'csrc')]


def _headers(directory):
    out = []
    for base, _, files in os.walk(directory):
        out += [os.path.join(base, f) for f in files
                if f.endswith(('.hpp', '.h'))]
    return out


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd, verbose):
    if verbose:
        print(' '.join(cmd), flush=True)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError('command failed: %s' % ' '.join(cmd[:3]))
    return proc.stdout


def compile_units(verbose=False, jobs=4):
    os.makedirs(OBJ, exist_ok=True)
    headers = _headers(os.path.join(ROOT, 'csrc'))
    units = []
    for sub in ('kernels', 'runtime'):
        d = os.path.join(ROOT, 'csrc', sub)
        for name in sorted(os.listdir(d)):
            if name.endswith(('.hip', '.cpp')):
                units.append(os.path.join(d, name))
    flags = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH,
             '-Wall', '-Wno-unused-result', '-Wno-unused-function',
             '-fvisibility=hidden'] + _includes()
    jobs_list = []
    for src in units:
        obj = os.path.join(OBJ, os.path.basename(src) + '.o')
        if _stale(obj, [src] + headers):
            cmd = [HIPCC] + flags + ['-c', src, '-o', obj]
            if src.endswith('.cpp'):
                cmd = [HIPCC] + flags + ['-x', 'hip', '-c', src, '-o', obj]
            jobs_list.append(cmd)
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as pool:
        list(pool.map(lambda c: _run(c, verbose), jobs_list))
    return [os.path.join(OBJ, os.path.basename(s) + '.o') for s in units]


def link_extension(objects, verbose=False):
    if not _stale(EXT_PATH, objects):
        return EXT_PATH
    cmd = [HIPCC, '-shared', '-fPIC', '--offload-arch=' + ARCH] + objects + \
        ['-o', EXT_PATH, '-ldl']
    _run(cmd, verbose)
    check_no_undefined_own_symbols(EXT_PATH)
    return EXT_PATH


def check_no_undefined_own_symbols(path):
    """The link cannot use --no-undefined (Python symbols resolve at import
    time), so a declaration/definition mismatch in our own code would only
    surface as an import error on the GPU box.  Fail the build instead."""
    nm = shutil.which('nm') or '/opt/rocm/lib/llvm/bin/llvm-nm'
    out = subprocess.run([nm, '-D', '-C', '--undefined-only', path],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True).stdout
    missing = [line.split()[-1] if '(' not in line else line.strip()
               for line in out.splitlines() if 'kiosk::' in line]
    if missing:
        os.remove(path)
        raise RuntimeError('undefined kiosk:: symbols in %s:\n  %s' % (
            path, '\n  '.join(missing)))


KREDIS_ASAN = os.path.join(BUILD, 'kredis-server-asan')
SANITIZE_FLAGS = ['-O1', '-g', '-fno-omit-frame-pointer',
                  '-fsanitize=address,undefined',
                  '-fno-sanitize-recover=undefined']


def build_kredis(verbose=False, sanitize=False):
    """``build/kredis-server`` (-O2), or with ``sanitize`` the ASan+UBSan
    build ``build/kredis-server-asan`` (the parser and network
    code is where memory bugs hide; tests/test_kredis_sanitized.py drives it
    with valid and malformed traffic)."""
    src_dir = os.path.join(ROOT, 'csrc', 'kredis')
    if not os.path.isdir(src_dir):
        return None
    sources = [os.path.join(src_dir, f) for f in sorted(os.listdir(src_dir))
               if f.endswith('.cpp')]
    if not sources:
        return None
    os.makedirs(BUILD, exist_ok=True)
    target = KREDIS_ASAN if sanitize else KREDIS
    flags = SANITIZE_FLAGS if sanitize else ['-O2']
    if _stale(target, sources + _headers(src_dir)):
        cxx = shutil.which('g++') or 'c++'
        _run([cxx] + flags + ['-std=c++17', '-Wall', '-pthread'] + sources +
             ['-o', target], verbose)
    return target


RCCL_SLIM_ASAN = os.path.join(BUILD, 'kiosk-rccl-slim-asan')


def build_rccl_slim(verbose=False, sanitize=False):
    """``build/kiosk-rccl-slim`` (g++, host only): writes the one-ISA,
    uncompressed, debug-stripped copy of RCCL the workers load
    (``parallel/rccl_lib.py``; csrc/tools/rccl_slim.cpp has the why).
    With ``sanitize`` the ASan+UBSan build ``build/kiosk-rccl-slim-asan``
    (it parses ELF and offload-bundle headers: tests/test_rccl_slim.py
    feeds it truncated and corrupted ones)."""
    src = os.path.join(ROOT, 'csrc', 'tools', 'rccl_slim.cpp')
    if not os.path.exists(src):
        return None
    os.makedirs(BUILD, exist_ok=True)
    target = RCCL_SLIM_ASAN if sanitize else RCCL_SLIM
    flags = SANITIZE_FLAGS if sanitize else ['-O2']
    if _stale(target, [src]):
        cxx = shutil.which('g++') or 'c++'
        _run([cxx] + flags + ['-std=c++17', '-Wall', src, '-o', target,
                              '-ldl'], verbose)
    return target


def build_fake(verbose=False):
    """CPU build of the node-communicator bindings over the fake HIP + RCCL
    (host code only: g++, no hipcc, no GPU)."""
    csrc = os.path.join(ROOT, 'csrc')
    runtime = os.path.join(csrc, 'runtime')
    fakes = os.path.join(csrc, 'fakes')
    os.makedirs(FAKE_DIR, exist_ok=True)
    cxx = shutil.which('g++') or 'c++'
    flags = ['-O2', '-g', '-std=c++17', '-fPIC', '-Wall', '-pthread',
             '-fvisibility=hidden', '-D__HIP_PLATFORM_AMD__',
             '-I/opt/rocm/include', '-I' + csrc, '-I' + runtime]
    lib_src = [os.path.join(fakes, 'fake_hip_rccl.cpp'),
               os.path.join(runtime, 'shmcomm.cpp')]
    headers = [os.path.join(runtime, h) for h in ('shmcomm.hpp', 'fence.hpp',
                                                  'bind_comm.hpp',
                                                  'trace.hpp', 'engine.hpp')]
    if _stale(FAKE_LIB, lib_src + headers):
        _run([cxx] + flags + ['-shared'] + lib_src + ['-o', FAKE_LIB],
             verbose)
    ext_src = [os.path.join(fakes, 'bind_cpu.cpp'),
               os.path.join(runtime, 'bind_comm.cpp'),
               os.path.join(runtime, 'fence.cpp'),
               os.path.join(runtime, 'trace.cpp'),
               os.path.join(runtime, 'shmcomm.cpp')]
    if _stale(FAKE_EXT, ext_src + headers + [FAKE_LIB]):
        _run([cxx] + flags + _includes() + ['-shared'] + ext_src +
             [FAKE_LIB, "-Wl,-rpath,$ORIGIN", '-ldl', '-o', FAKE_EXT],
             verbose)
    return FAKE_EXT


def build(verbose=False, clean=False, jobs=4, kernels=True, sanitize=False,
          fake=True):
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    out = {'kredis': build_kredis(verbose),
           'rccl_slim': build_rccl_slim(verbose)}
    if fake:
        out['fake_fence'] = build_fake(verbose)
    if sanitize:
        out['kredis_asan'] = build_kredis(verbose, sanitize=True)
        out['rccl_slim_asan'] = build_rccl_slim(verbose, sanitize=True)
    if kernels:
        objects = compile_units(verbose, jobs)
        out['extension'] = link_extension(objects, verbose)
    return out


def main():
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('-v', '--verbose', action='store_true')
    parser.add_argument('--clean', action='store_true')
    parser.add_argument('-j', '--jobs', type=int, default=4)
    parser.add_argument('--no-kernels', action='store_true')
    parser.add_argument('--sanitize', action='store_true',
                        help='also build the ASan+UBSan kredis-server and '
                             'kiosk-rccl-slim')
    parser.add_argument('--fake-hip', action='store_true',
                        help='only the CPU fence module over the fake '
                             'HIP + RCCL (build/fake)')
    args = parser.parse_args()
    if args.fake_hip:
        print('fake_fence: %s' % build_fake(args.verbose))
        return
    out = build(args.verbose, args.clean, args.jobs, not args.no_kernels,
                args.sanitize)
    for key, value in out.items():
        print('%s: %s' % (key, value))


if __name__ == '__main__':
    main()
