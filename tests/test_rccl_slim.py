"""The one-ISA RCCL copy (``csrc/tools/rccl_slim.cpp``,
``parallel/rccl_lib.py``): bundle parsing, streamed zstd inflation, DWARF
stripping, the in-place section rewrite, the cache, and on MI355X that the
copy drives a real RCCL generation.

CPU cases build a small ELF shared library with a ``.hip_fatbin`` section
holding a zstd-compressed (CCOB v3) or plain offload bundle of fake code
objects; one case slims ROCm's own librccl when the image has it."""
import ctypes
import json
import os
import struct
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

from kiosk_autoscaler_amd.parallel import rccl_lib  # noqa: E402

MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


@pytest.fixture(scope='module')
def tool():
    import build_native
    path = build_native.build_rccl_slim()
    if path is None or not os.path.exists(path):
        pytest.skip('kiosk-rccl-slim not built')
    return path


def _cc(args):
    cc = 'gcc'
    subprocess.run([cc] + args, check=True, capture_output=True)


def _code_object(tmp, name, body):
    """A shared object with DWARF (stands in for a gfx code object)."""
    src = os.path.join(tmp, name + '.c')
    with open(src, 'w') as f:
        f.write('int %s_fn(int x) { return x * %d + 1; }\n'
                'const char %s_tag[] = "%s";\n' % (name, body, name, name))
    out = os.path.join(tmp, name + '.so')
    _cc(['-shared', '-fPIC', '-g', '-O1', src, '-o', out])
    with open(out, 'rb') as f:
        return f.read()


def _bundle(entries):
    """An uncompressed clang offload bundle of ``[(id, bytes)]``."""
    header = MAGIC + struct.pack('<Q', len(entries))
    size = len(header) + sum(24 + len(i) for i, _ in entries)
    offset = (size + 4095) // 4096 * 4096
    table, blobs = b'', b''
    for ident, blob in entries:
        if blob:
            pad = (-(offset + len(blobs))) % 4096
            blobs += b'\0' * pad
        table += struct.pack('<QQQ', offset + len(blobs), len(blob),
                             len(ident)) + ident.encode()
        blobs += blob
    head = header + table
    return head + b'\0' * (offset - len(head)) + blobs


def _ccob(bundle):
    zstd = ctypes.CDLL('libzstd.so.1')
    zstd.ZSTD_compressBound.restype = ctypes.c_size_t
    zstd.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    zstd.ZSTD_compress.restype = ctypes.c_size_t
    zstd.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.c_int]
    cap = zstd.ZSTD_compressBound(len(bundle))
    out = ctypes.create_string_buffer(cap)
    n = zstd.ZSTD_compress(out, cap, bundle, len(bundle), 3)
    payload = out.raw[:n]
    header = b'CCOB' + struct.pack('<HHQQQ', 3, 1, 32 + n, len(bundle), 0)
    return header + payload


def _library(tmp, fatbin, slack=1 << 16):
    """A shared library whose ``.hip_fatbin`` section holds ``fatbin``
    (padded, as a real one is larger than any slim bundle)."""
    size = len(fatbin) + slack
    src = os.path.join(tmp, 'lib.c')
    with open(src, 'w') as f:
        f.write('__attribute__((section(".hip_fatbin"), used, aligned(4096)))\n'
                'const unsigned char fatbin[%d] = {1};\n'
                'int ncclGetVersion(int* v) { *v = 22707; return 0; }\n'
                % size)
    lib = os.path.join(tmp, 'librccl.so.1')
    _cc(['-shared', '-fPIC', src, '-o', lib])
    sec_off, sec_size = _section(lib, '.hip_fatbin')
    assert sec_size == size
    with open(lib, 'r+b') as f:
        f.seek(sec_off)
        f.write(fatbin + b'\0' * (sec_size - len(fatbin)))
    return lib


def _section(path, name):
    with open(path, 'rb') as f:
        data = f.read()
    shoff, = struct.unpack_from('<Q', data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', data, 0x3a)
    sections = [struct.unpack_from('<IIQQQQIIQQ', data, shoff + i * shentsize)
                for i in range(shnum)]
    stroff = sections[shstrndx][4]
    for sh in sections:
        end = data.index(b'\0', stroff + sh[0])
        if data[stroff + sh[0]:end].decode() == name:
            return sh[4], sh[5]
    raise KeyError(name)


def _parse_bundle(blob):
    assert blob[:24] == MAGIC
    n, = struct.unpack_from('<Q', blob, 24)
    pos, out = 32, {}
    for _ in range(n):
        off, size, idlen = struct.unpack_from('<QQQ', blob, pos)
        pos += 24
        ident = blob[pos:pos + idlen].decode()
        pos += idlen
        out[ident] = blob[off:off + size]
    return out


def _sections_of(blob):
    shoff, = struct.unpack_from('<Q', blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', blob, 0x3a)
    secs = [struct.unpack_from('<IIQQQQIIQQ', blob, shoff + i * shentsize)
            for i in range(shnum)]
    stroff = secs[shstrndx][4]
    names = []
    for sh in secs:
        end = blob.index(b'\0', stroff + sh[0])
        names.append(blob[stroff + sh[0]:end].decode())
    return names, secs


@pytest.mark.parametrize('compressed', [True, False])
def test_slim_keeps_one_isa_uncompressed_and_stripped(tmp_path, tool,
                                                      compressed):
    tmp = str(tmp_path)
    gfx942 = _code_object(tmp, 'k942', 3)
    gfx950 = _code_object(tmp, 'k950', 5)
    bundle = _bundle([('host-x86_64-unknown-linux-gnu-', b''),
                      ('hipv4-amdgcn-amd-amdhsa--gfx942:xnack-', gfx942),
                      ('hipv4-amdgcn-amd-amdhsa--gfx950:xnack+', gfx942),
                      ('hipv4-amdgcn-amd-amdhsa--gfx950', gfx950)])
    fatbin = _ccob(bundle) if compressed else bundle
    lib = _library(tmp, fatbin, slack=len(bundle))
    out = os.path.join(tmp, 'slim', 'librccl.so.1')
    os.makedirs(os.path.dirname(out))
    proc = subprocess.run([tool, '--src', lib, '--out', out], check=True,
                          capture_output=True, text=True)
    info = json.loads(proc.stdout)
    assert info['compressed'] is compressed
    assert info['entry'] == 'hipv4-amdgcn-amd-amdhsa--gfx950'   # not xnack+
    assert info['code_object_bytes'] == len(gfx950)
    # the library keeps its size and layout: only the section changed
    assert os.path.getsize(out) == os.path.getsize(lib)
    with open(lib, 'rb') as f:
        old = f.read()
    with open(out, 'rb') as f:
        new = f.read()
    sec_off, sec_size = _section(out, '.hip_fatbin')
    assert new[:sec_off] == old[:sec_off]
    assert new[sec_off + sec_size:] == old[sec_off + sec_size:]
    entries = _parse_bundle(new[sec_off:sec_off + sec_size])
    assert set(entries) == {'host-x86_64-unknown-linux-gnu-',
                            'hipv4-amdgcn-amd-amdhsa--gfx950'}
    code = entries['hipv4-amdgcn-amd-amdhsa--gfx950']
    assert len(code) == info['slim_code_object_bytes'] < len(gfx950)
    names, secs = _sections_of(code)
    assert not [n for n in names if n.startswith('.debug')]
    old_names, old_secs = _sections_of(gfx950)
    assert [n for n in old_names if n.startswith('.debug')]
    # every allocated section is byte-identical, at the same offset
    for name, sh in zip(old_names, old_secs):
        if sh[2] & 0x2 and sh[1] != 8:      # SHF_ALLOC, not NOBITS
            i = names.index(name)
            assert secs[i][4] == sh[4]
            assert code[sh[4]:sh[4] + sh[5]] == gfx950[sh[4]:sh[4] + sh[5]]
    # the stripped object is still a valid shared object for the loader
    stripped = os.path.join(tmp, 'stripped.so')
    with open(stripped, 'wb') as f:
        f.write(code)
    lib_co = ctypes.CDLL(stripped)
    assert lib_co.k950_fn(2) == 11
    assert ctypes.CDLL(out).ncclGetVersion(ctypes.byref(ctypes.c_int())) == 0


@pytest.fixture(scope='module')
def asan_tool():
    import build_native
    try:
        path = build_native.build_rccl_slim(sanitize=True)
    except Exception as err:  # pylint: disable=broad-except
        pytest.skip('no sanitizer build: %s' % err)
    if path is None or not os.path.exists(path):
        pytest.skip('kiosk-rccl-slim-asan not built')
    return path


# size fields the tool bounds by the section instead of trusting: a bogus
# value leaves the result intact
_TOLERATED = ('ccob_total_huge', 'ccob_inflated_huge')


def _corruptions(lib):
    """Truncated and corrupted copies of a good library: the tool must
    refuse each (exit 2) without reading out of bounds, or -- for a size
    field it bounds itself (``_TOLERATED``) -- still slim it."""
    with open(lib, 'rb') as f:
        good = f.read()
    sec_off, sec_size = _section(lib, '.hip_fatbin')
    out = {'empty': b'', 'elf_header_only': good[:64],
           'cut_before_section': good[:sec_off + 16],
           'cut_in_section': good[:sec_off + sec_size // 2]}
    shoff, = struct.unpack_from('<Q', good, 0x28)

    def patched(offset, fmt, value):
        blob = bytearray(good)
        struct.pack_into(fmt, blob, offset, value)
        return bytes(blob)
    out['shoff_past_eof'] = patched(0x28, '<Q', len(good) + 4096)
    out['shnum_huge'] = patched(0x3c, '<H', 0xfff0)
    out['shstrndx_bad'] = patched(0x3e, '<H', 0xfff0)
    body = sec_off
    if good[body:body + 4] == b'CCOB':
        out['ccob_total_huge'] = patched(body + 8, '<Q', 1 << 60)
        out['ccob_inflated_huge'] = patched(body + 16, '<Q', 1 << 60)
        out['ccob_payload_garbage'] = patched(body + 32, '<Q',
                                              0x4141414141414141)
        out['ccob_version_9'] = patched(body + 4, '<H', 9)
    else:
        out['bundle_count_huge'] = patched(body + 24, '<Q', 1 << 40)
        # the gfx950 entry's offset / size, and an id length past the table
        pos = body + 32
        count, = struct.unpack_from('<Q', good, body + 24)
        for _ in range(count):
            _, size, idlen = struct.unpack_from('<QQQ', good, pos)
            if size:
                break
            pos += 24 + idlen
        out['entry_offset_past_end'] = patched(pos, '<Q', 1 << 40)
        out['entry_size_huge'] = patched(pos + 8, '<Q', 1 << 40)
        out['entry_offset_wraps'] = patched(pos, '<Q', (1 << 64) - 16)
        out['entry_idlen_huge'] = patched(body + 48, '<Q', 1 << 40)
    return out


@pytest.mark.parametrize('compressed', [True, False])
def test_sanitized_slim_survives_malformed_libraries(tmp_path, asan_tool,
                                                     compressed):
    """SURVEY §5.2 for the new parser: under ASan+UBSan the tool slims a
    good library and refuses truncated / corrupted ELF and bundle headers
    cleanly (exit 2, no sanitizer report)."""
    tmp = str(tmp_path)
    bundle = _bundle([('host-x86_64-unknown-linux-gnu-', b''),
                      ('hipv4-amdgcn-amd-amdhsa--gfx950',
                       _code_object(tmp, 'k950', 5))])
    lib = _library(tmp, _ccob(bundle) if compressed else bundle,
                   slack=len(bundle))
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:exitcode=99',
               UBSAN_OPTIONS='halt_on_error=1:exitcode=98')
    ok = subprocess.run([asan_tool, '--src', lib, '--out',
                         os.path.join(tmp, 'ok.so')], env=env,
                        capture_output=True, text=True, timeout=120)
    assert ok.returncode == 0, ok.stderr[-2000:]
    for name, blob in _corruptions(lib).items():
        bad = os.path.join(tmp, 'bad_%s.so' % name)
        with open(bad, 'wb') as f:
            f.write(blob)
        proc = subprocess.run([asan_tool, '--src', bad, '--out',
                               os.path.join(tmp, 'out_%s.so' % name)],
                              env=env, capture_output=True, text=True,
                              timeout=120)
        assert 'Sanitizer' not in proc.stderr, (name, proc.stderr[-3000:])
        want = 0 if name in _TOLERATED else 2
        assert proc.returncode == want, (name, proc.returncode,
                                         proc.stderr[-2000:])


def _code_object_corruptions(code):
    """Corrupted copies of a gfx950 code object (the debug
    stripper trusted the object's program-header, section and name
    offsets)."""
    shoff, = struct.unpack_from('<Q', code, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', code, 0x3a)

    def patched(offset, fmt, value):
        blob = bytearray(code)
        struct.pack_into(fmt, blob, offset, value)
        return bytes(blob)
    names, secs = _sections_of(code)
    debug = next(i for i, n in enumerate(names) if n.startswith('.debug'))
    sec = shoff + debug * shentsize
    strsec = shoff + shstrndx * shentsize
    return {
        'phoff_past_end': patched(0x20, '<Q', len(code) + 4096),
        'phnum_huge': patched(0x38, '<H', 0xfff0),
        'section_offset_past_end': patched(sec + 0x18, '<Q', 1 << 40),
        'section_size_huge': patched(sec + 0x20, '<Q', 1 << 40),
        'section_name_past_strtab': patched(sec, '<I', 0xffffff00),
        'strtab_size_huge': patched(strsec + 0x20, '<Q', 1 << 40),
    }


def test_sanitized_slim_refuses_corrupted_code_objects(tmp_path, asan_tool):
    """The gfx950 code object itself corrupted: the stripper refuses it
    (exit 2) without an out-of-bounds read under ASan+UBSan."""
    tmp = str(tmp_path)
    code = _code_object(tmp, 'k950', 5)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:exitcode=99',
               UBSAN_OPTIONS='halt_on_error=1:exitcode=98')
    for name, blob in _code_object_corruptions(code).items():
        bundle = _bundle([('host-x86_64-unknown-linux-gnu-', b''),
                          ('hipv4-amdgcn-amd-amdhsa--gfx950', blob)])
        sub = os.path.join(tmp, name)
        os.makedirs(sub)
        lib = _library(sub, bundle, slack=len(bundle))
        proc = subprocess.run([asan_tool, '--src', lib, '--out',
                               os.path.join(sub, 'out.so')], env=env,
                              capture_output=True, text=True, timeout=120)
        assert 'Sanitizer' not in proc.stderr, (name, proc.stderr[-3000:])
        # a name past the string table reads as empty (bounded): that
        # section is kept, the object is still slimmed
        want = 0 if name == 'section_name_past_strtab' else 2
        assert proc.returncode == want, (name, proc.returncode,
                                         proc.stderr[-2000:])


def test_slim_cache_key_follows_the_tool(tmp_path, tool):
    """a copy written by an earlier build of the tool is not
    loaded after the tool changes (its content hash is in the key)."""
    import shutil
    tmp = str(tmp_path)
    other = os.path.join(tmp, 'tool-copy')
    shutil.copy(tool, other)
    lib = os.path.join(tmp, 'lib.so')
    with open(lib, 'wb') as f:
        f.write(b'x')
    same = rccl_lib.slim_dir(lib, tool=other) == rccl_lib.slim_dir(lib,
                                                                    tool=tool)
    assert same
    with open(other, 'ab') as f:
        f.write(b'rebuilt')
    assert rccl_lib.slim_dir(lib, tool=other) != rccl_lib.slim_dir(lib,
                                                                    tool=tool)


def test_slim_refuses_a_bundle_without_the_isa(tmp_path, tool):
    tmp = str(tmp_path)
    bundle = _bundle([('host-x86_64-unknown-linux-gnu-', b''),
                      ('hipv4-amdgcn-amd-amdhsa--gfx942',
                       _code_object(tmp, 'k942', 3))])
    lib = _library(tmp, _ccob(bundle))
    proc = subprocess.run([tool, '--src', lib, '--out',
                           os.path.join(tmp, 'x.so')],
                          capture_output=True, text=True)
    assert proc.returncode == 2
    assert 'no gfx950 entry' in proc.stderr
    assert not os.path.exists(os.path.join(tmp, 'x.so'))


def test_ensure_slim_caches_and_configure_exports(tmp_path, tool):
    tmp = str(tmp_path)
    bundle = _bundle([('host-x86_64-unknown-linux-gnu-', b''),
                      ('hipv4-amdgcn-amd-amdhsa--gfx950',
                       _code_object(tmp, 'k950', 5))])
    lib = _library(tmp, _ccob(bundle))
    env = {'KIOSK_CACHE_DIR': os.path.join(tmp, 'cache'),
           'KIOSK_RCCL_SRC': lib}
    path, info = rccl_lib.ensure_slim(env=env, tool=tool)
    assert path and os.path.exists(path) and info['cached'] is False
    again, info2 = rccl_lib.ensure_slim(env=env, tool=tool)
    assert again == path and info2['cached'] is True
    assert rccl_lib.cached(env=env) == path
    # configure(): exported for every process the manager spawns
    env2 = dict(env)
    out = rccl_lib.configure(env=env2)
    assert out['slim'] and env2['KIOSK_RCCL_LIB'] == path
    # an operator's explicit library wins; RCCL_SLIM=0 opts out
    env3 = dict(env, KIOSK_RCCL_LIB='/x/librccl.so.1')
    assert rccl_lib.configure(env=env3)['slim'] is False
    assert env3['KIOSK_RCCL_LIB'] == '/x/librccl.so.1'
    env4 = dict(env, RCCL_SLIM='0')
    assert rccl_lib.configure(env=env4)['slim'] is False
    assert 'KIOSK_RCCL_LIB' not in env4
    # a source that changes gets a new copy (the key covers size + mtime)
    os.utime(lib, ns=(1, 1))
    assert rccl_lib.cached(env=env) is None


def test_configure_falls_back_to_stock_without_the_tool(tmp_path):
    env = {'KIOSK_CACHE_DIR': str(tmp_path), 'KIOSK_RCCL_SRC': '/nonexistent'}
    out = rccl_lib.configure(env=env)
    assert out['slim'] is False and 'KIOSK_RCCL_LIB' not in env
    assert out.get('error')


@pytest.mark.skipif(not os.path.exists(rccl_lib.STOCK),
                    reason='no ROCm RCCL in this image')
def test_slim_rocm_rccl(tmp_path, tool):
    """ROCm 7.2's librccl: 13 targets, 5.3 GB inflated, gfx950 last."""
    out = os.path.join(str(tmp_path), 'librccl.so.1')
    proc = subprocess.run([tool, '--src', rccl_lib.STOCK, '--out', out],
                          check=True, capture_output=True, text=True,
                          timeout=300)
    info = json.loads(proc.stdout)
    assert info['compressed'] and info['entry'].endswith('--gfx950')
    assert info['inflated_bytes'] > 4 << 30
    assert info['slim_code_object_bytes'] < info['code_object_bytes'] / 4
    # the copy is sparse: the unused tail of the section is a hole
    assert os.stat(out).st_blocks * 512 < os.path.getsize(out) / 2
    version = ctypes.c_int()
    assert ctypes.CDLL(out).ncclGetVersion(ctypes.byref(version)) == 0
    assert version.value >= 22700


_GENERATION = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
from kiosk_autoscaler_amd.ops import native
mod = native.load(torch_first=False)
mod.preinit_device(0)
import time
t0 = time.perf_counter()
fence = mod.Fence(mod.fence_unique_id(), 1, 0, 60.0)
init_ms = (time.perf_counter() - t0) * 1e3
result, us = fence.allreduce([3, 0, 1, 0, 0, 0, 0, 0, 0])
fence.destroy()
print(json.dumps({'lib': mod.rccl_library(), 'init_ms': init_ms,
                  'result': list(result)}))
'''


@pytest.mark.gpu
def test_gpu_slim_rccl_generation():
    """The slim copy drives a real 1-rank RCCL generation on MI355X, and
    its first init is far cheaper than the stock library's (no 5.3 GB
    inflation; profiles/r5_fence_lag)."""
    path, info = rccl_lib.ensure_slim()
    assert path, info
    env = dict(os.environ, KIOSK_RCCL_LIB=path, NCCL_MIN_NCHANNELS='1',
               NCCL_MAX_NCHANNELS='1')
    proc = subprocess.run([sys.executable, '-c', _GENERATION, ROOT],
                          capture_output=True, text=True, timeout=120,
                          env=env)
    assert proc.returncode == 0, proc.stderr[-2000:]
    row = json.loads(proc.stdout.strip().splitlines()[-1])
    assert row['lib'] == path
    assert row['result'] == [3, 0, 1, 0, 0, 0, 0, 0, 0]
    assert row['init_ms'] < 1500, row
