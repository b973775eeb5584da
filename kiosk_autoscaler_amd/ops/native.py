"""Loader for the in-tree native module ``_kiosk_hip`` (HIP/gfx950 + RCCL).

Load order matters: PyTorch-ROCm bundles its own ``libamdhip64.so`` (SONAME
``libamdhip64.so.7``).  In a process that uses torch, importing torch first
makes the extension's ``libamdhip64.so.7`` dependency resolve to that
already-loaded runtime, so one HIP runtime serves both (two runtimes in one
process would each own the device).  The worker never uses torch: it loads
the extension with ``torch_first=False`` and runs on ROCm's own runtime (the
one the extension was compiled against), which takes the ~1.5 s torch
import -- minutes on a fresh node -- off standby boot and cold spawns.
A torch process gets ROCm's own code-object compiler (comgr) instead of
torch's bundled copy (:func:`prefer_rocm_comgr`): the HIP runtime compiles
its blit kernels through comgr when the process creates its first stream,
and torch's comgr caches only the back half of that compile, so every
PyTorch standby paid ~60 ms of OpenCL front end at boot
(``profiles/r4_stream``).
RCCL is *not* a link-time dependency: the fence code ``dlopen``s a full RCCL
(``KIOSK_RCCL_LIB``, default ROCm's, which has ``ncclCommShrink``) with
``RTLD_LOCAL``.

There is no silent fallback: on a machine with a GPU a missing or stale
extension raises :class:`NativeUnavailable` with the build command.

``KIOSK_NATIVE=fake`` (CPU tests only) loads ``build/fake/_kiosk_fence_cpu``
instead: the same node-communicator bindings (RCCL ``Fence``, ``ShmComm``)
compiled for the host against the shared-memory fake HIP + RCCL
(``tools/build_native.py --fake-hip``), so the production fence path runs in
N CPU processes.  It has no kernels and no engine.
"""
import ctypes
import glob
import importlib
import os
import sys

_MOD = None
HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_HINT = ('build it with `python tools/build_native.py` '
              '(or `python -c "import __graft_entry__ as g; g.build()"`)')


class NativeUnavailable(ImportError):
    pass


ROOT = os.path.dirname(os.path.dirname(HERE))
FAKE_DIR = os.path.join(ROOT, 'build', 'fake')


def extension_candidates():
    return sorted(glob.glob(os.path.join(HERE, '_kiosk_hip*.so')))


def fake_requested():
    return os.environ.get('KIOSK_NATIVE', '') == 'fake'


def _load_fake():
    paths = sorted(glob.glob(os.path.join(FAKE_DIR, '_kiosk_fence_cpu*.so')))
    if not paths:
        raise NativeUnavailable('KIOSK_NATIVE=fake but build/fake is not '
                                'built; run `python tools/build_native.py '
                                '--fake-hip`')
    # the fence dlopen()s RCCL: point it at the fake (already mapped as the
    # module's dependency, so both resolve to one library)
    os.environ.setdefault('KIOSK_RCCL_LIB', os.path.join(
        FAKE_DIR, 'libkiosk_fake_hip_rccl.so'))
    if FAKE_DIR not in sys.path:
        sys.path.insert(0, FAKE_DIR)
    return importlib.import_module('_kiosk_fence_cpu')


def elf_soname(path):
    """``DT_SONAME`` of an ELF64 shared library, or None."""
    import struct
    try:
        with open(path, 'rb') as f:
            head = f.read(64)
            if head[:4] != b'\x7fELF' or head[4] != 2:
                return None
            shoff, = struct.unpack_from('<Q', head, 0x28)
            shentsize, shnum = struct.unpack_from('<HH', head, 0x3a)
            f.seek(shoff)
            table = f.read(shentsize * shnum)
            sections = [struct.unpack_from('<IIQQQQIIQQ', table, i * shentsize)
                        for i in range(shnum)]
            for sh in sections:
                if sh[1] != 6:                    # SHT_DYNAMIC
                    continue
                f.seek(sh[4])
                dyn = f.read(sh[5])
                strtab = sections[sh[6]]
                for off in range(0, len(dyn) - 15, 16):
                    tag, val = struct.unpack_from('<qQ', dyn, off)
                    if tag == 14:                 # DT_SONAME
                        f.seek(strtab[4] + val)
                        return f.read(256).split(b'\0')[0].decode()
    except (OSError, IndexError, struct.error, UnicodeDecodeError):
        return None
    return None


def comgr_abi_matches(torch_lib=None, rocm_lib='/opt/rocm/lib/libamd_comgr.so'):
    """True when ROCm's comgr has the soname (ABI major) of the copy torch
    bundles -- the one its HIP runtime was linked against.  Found without
    importing torch (its package directory is located by name)."""
    if torch_lib is None:
        import importlib.util
        spec = importlib.util.find_spec('torch')
        if spec is None or not spec.submodule_search_locations:
            return False
        torch_lib = os.path.join(list(spec.submodule_search_locations)[0],
                                 'lib', 'libamd_comgr.so')
    ours, theirs = elf_soname(os.path.realpath(rocm_lib)), \
        elf_soname(torch_lib)
    return ours is not None and ours == theirs


def prefer_rocm_comgr():
    """Map ROCm's ``libamd_comgr.so`` before torch loads its own.

    Torch's ``libamdhip64.so`` needs ``libamd_comgr.so`` (unversioned) via
    an ``$ORIGIN`` RPATH.  A library already loaded *under that name* meets
    the dependency, so a bare-name ``dlopen`` (resolved by the loader cache
    to ``/opt/rocm``) puts ROCm 7.2's comgr under torch's HIP runtime; the
    HIP and HSA runtimes stay torch's own (one of each per process).
    ROCm's comgr caches the whole blit-kernel compile on disk
    (``AMD_COMGR_CACHE``, on by default), torch's 7.0 copy only its code
    generation: a torch process's first stream drops from ~85 ms to
    ~20 ms.  No-op once torch is imported, with
    ``KIOSK_TORCH_COMGR=bundled`` (keep torch's copy), or when ROCm's comgr
    has another soname (ABI major) than torch's bundled one; returns the
    path mapped, or None."""
    if 'torch' in sys.modules or \
            os.environ.get('KIOSK_TORCH_COMGR') == 'bundled':
        return None
    if not comgr_abi_matches():
        # another comgr ABI than the one torch's HIP runtime was built
        # against: keep torch's bundled copy
        return None
    try:
        ctypes.CDLL('libamd_comgr.so', mode=ctypes.RTLD_GLOBAL)
    except OSError:
        return None
    try:
        with open('/proc/self/maps') as maps:
            paths = {line.split()[-1] for line in maps if 'comgr' in line}
    except OSError:
        return None
    return sorted(paths)[0] if paths else None


def load(torch_first=True):
    """Import and return the native module (cached; the first call decides
    the load order).  ``torch_first=False`` is for processes that never
    import torch (the worker)."""
    global _MOD
    if _MOD is not None:
        return _MOD
    if fake_requested():
        _MOD = _load_fake()
        return _MOD
    if not extension_candidates():
        raise NativeUnavailable('native module _kiosk_hip is not built; '
                                + BUILD_HINT)
    if torch_first:
        prefer_rocm_comgr()
        try:
            import torch  # noqa: F401  -- must precede the extension
        except ImportError:
            pass
    try:
        _MOD = importlib.import_module('kiosk_autoscaler_amd.ops._kiosk_hip')
    except ImportError as err:
        raise NativeUnavailable('cannot import _kiosk_hip (%s); %s' % (
            err, BUILD_HINT))
    return _MOD


def available():
    try:
        load()
        return True
    except NativeUnavailable:
        return False


def loaded_path():
    mod = sys.modules.get('kiosk_autoscaler_amd.ops._kiosk_hip') or \
        sys.modules.get('_kiosk_fence_cpu')
    return getattr(mod, '__file__', None)
