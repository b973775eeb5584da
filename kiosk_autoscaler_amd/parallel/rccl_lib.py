"""Which RCCL library the node communicator loads.

The fence ``dlopen``s RCCL (``csrc/runtime/fence.cpp``, ``KIOSK_RCCL_LIB``).
ROCm's stock ``librccl.so.1`` carries its device code for thirteen GPU
targets in one zstd-compressed offload bundle that inflates to 5.3 GB, with
gfx950 last.  The HIP runtime digests a fat binary lazily, in the first
``ncclCommInitRank`` of each process, so every freshly forked worker paid
~1.1 s of decompression plus a 569 MB code-object load in its first
generation (the fenced set trailed READY by 1.75 s).

:func:`ensure_slim` writes, once per host and source library, a copy whose
fat binary holds only the gfx950 code object, uncompressed and without its
DWARF (108 MB; ``build/kiosk-rccl-slim``, ``csrc/tools/rccl_slim.cpp``).  The
manager calls it at start and points its workers at the copy
(``RCCL_SLIM``, default on for the RCCL fence).  The copy lives in a cache
directory (``KIOSK_CACHE_DIR``, default ``~/.cache/kiosk-autoscaler-amd``)
beside a ``share/rccl`` link, so RCCL still finds its MSCCL algorithm files
relative to itself.
"""
import fcntl
import hashlib
import json
import logging
import os
import subprocess
import time

logger = logging.getLogger('RcclLib')

STOCK = '/opt/rocm/lib/librccl.so.1'
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
TOOL = os.path.join(ROOT, 'build', 'kiosk-rccl-slim')
MANIFEST = 'slim.json'


def cache_root(env=None):
    env = os.environ if env is None else env
    base = env.get('KIOSK_CACHE_DIR')
    if not base:
        home = env.get('XDG_CACHE_HOME') or os.path.join(
            os.path.expanduser('~'), '.cache')
        base = os.path.join(home, 'kiosk-autoscaler-amd')
    return base


def source_library(env=None):
    """The RCCL the slim copy is made from: ``KIOSK_RCCL_SRC``, else ROCm's
    (its ``ncclCommShrink`` is what the node communicator needs)."""
    env = os.environ if env is None else env
    return os.path.realpath(env.get('KIOSK_RCCL_SRC') or STOCK)


# bumped whenever the slim copy's layout changes (a copy made
# by an earlier, buggy tool must not be loaded after the tool is fixed)
FORMAT_VERSION = 2


def _tool_id(tool=None):
    """Content hash of the slimming tool: a rebuilt tool makes a new copy."""
    tool = tool or TOOL
    try:
        with open(tool, 'rb') as handle:
            return hashlib.sha1(handle.read()).hexdigest()[:12]
    except OSError:
        return 'none'


def _key(src, isa, strip, tool=None):
    st = os.stat(src)
    text = '%s|%d|%d|%s|%d|v%d|%s' % (src, st.st_size, st.st_mtime_ns, isa,
                                      int(strip), FORMAT_VERSION,
                                      _tool_id(tool))
    return hashlib.sha1(text.encode()).hexdigest()[:16]


def slim_dir(src, isa='gfx950', strip=True, env=None, tool=None):
    return os.path.join(cache_root(env), 'rccl-%s-%s' % (
        isa, _key(src, isa, strip, tool)))


def _link_share(target_dir, src):
    """``<dir>/share/rccl`` -> the source install's, for the paths RCCL
    resolves relative to its own file (``../share/rccl/msccl-algorithms``)."""
    share = os.path.normpath(os.path.join(os.path.dirname(src), '..',
                                          'share', 'rccl'))
    if not os.path.isdir(share):
        return
    os.makedirs(os.path.join(target_dir, 'share'), exist_ok=True)
    link = os.path.join(target_dir, 'share', 'rccl')
    if not os.path.lexists(link):
        try:
            os.symlink(share, link)
        except OSError:
            pass


def cached(src=None, isa='gfx950', strip=True, env=None):
    """The slim library's path if it was already written, else None."""
    src = src or source_library(env)
    try:
        directory = slim_dir(src, isa, strip, env)
    except OSError:
        return None
    path = os.path.join(directory, 'lib', 'librccl.so.1')
    manifest = os.path.join(directory, MANIFEST)
    if os.path.exists(path) and os.path.exists(manifest):
        return path
    return None


def ensure_slim(src=None, isa='gfx950', strip=True, env=None, tool=None,
                timeout=300.0):
    """Path of the slim RCCL for ``isa``, writing it first if needed (one
    writer per host: an flock on the cache directory).  Returns
    ``(path, info)``; ``(None, info)`` when it cannot be made -- the caller
    keeps the stock library, ``info['error']`` says why."""
    src = src or source_library(env)
    tool = tool or TOOL
    t0 = time.monotonic()
    try:
        directory = slim_dir(src, isa, strip, env, tool)
    except OSError as err:
        return None, {'error': 'source RCCL: %s' % err, 'src': src}
    path = os.path.join(directory, 'lib', 'librccl.so.1')
    manifest = os.path.join(directory, MANIFEST)
    try:
        os.makedirs(os.path.join(directory, 'lib'), exist_ok=True)
    except OSError as err:
        return None, {'error': 'cache dir: %s' % err, 'src': src}
    with open(os.path.join(directory, '.lock'), 'w') as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if os.path.exists(path) and os.path.exists(manifest):
            try:
                with open(manifest) as f:
                    info = json.load(f)
            except (OSError, ValueError):
                info = {}
            info['cached'] = True
            info['ms'] = (time.monotonic() - t0) * 1e3
            return path, info
        if not os.path.exists(tool):
            return None, {'error': 'tool not built: %s' % tool, 'src': src}
        cmd = [tool, '--src', src, '--out', path, '--isa', isa]
        if not strip:
            cmd.append('--no-strip')
        try:
            proc = subprocess.run(cmd, stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True,
                                  timeout=timeout)
        except (OSError, subprocess.TimeoutExpired) as err:
            return None, {'error': str(err), 'src': src}
        if proc.returncode != 0:
            return None, {'error': proc.stderr.strip()[-500:] or
                          'exit %d' % proc.returncode, 'src': src}
        try:
            info = json.loads(proc.stdout.strip().splitlines()[-1])
        except (ValueError, IndexError):
            info = {}
        _link_share(directory, src)
        with open(manifest + '.tmp', 'w') as f:
            json.dump(info, f)
        os.replace(manifest + '.tmp', manifest)
        info['cached'] = False
        info['ms'] = (time.monotonic() - t0) * 1e3
        return path, info


def configure(env=None, isa=None, log=None):
    """Manager start: unless ``KIOSK_RCCL_LIB`` already names a library or
    ``RCCL_SLIM=0``, make (or find) the slim copy and export it as
    ``KIOSK_RCCL_LIB`` into ``env`` (default ``os.environ``), which every
    zygote, standby and worker inherits.  Returns the info dict."""
    env = os.environ if env is None else env
    log = log or logger
    if env.get('KIOSK_RCCL_LIB'):
        return {'lib': env['KIOSK_RCCL_LIB'], 'slim': False,
                'reason': 'KIOSK_RCCL_LIB set'}
    if str(env.get('RCCL_SLIM', '1')).lower() in ('0', 'false', 'no', 'off'):
        return {'lib': None, 'slim': False, 'reason': 'RCCL_SLIM=0'}
    isa = isa or env.get('KIOSK_OFFLOAD_ARCH') or 'gfx950'
    path, info = ensure_slim(isa=isa, env=env)
    if path is None:
        log.warning('slim RCCL unavailable (%s): workers load the stock '
                    'library.', info.get('error'))
        return dict(info, lib=None, slim=False)
    env['KIOSK_RCCL_LIB'] = path
    log.info('RCCL for the node communicator: %s (%s, %.0f ms%s).', path,
             info.get('entry', isa), info.get('ms', 0.0),
             ', cached' if info.get('cached') else '')
    return dict(info, lib=path, slim=True)
