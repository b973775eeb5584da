"""csrc/runtime/fence.cpp under AddressSanitizer + UBSan, and under
ThreadSanitizer, on the host (CPU):
the fence's failure paths -- async init error, init timeout, abort
requested before connect or during an all-reduce blocked on a dead peer,
all-reduce timeout, stuck finalize, a rank dying mid-all-reduce and the
survivors shrinking it out (NCCL_SHRINK_ABORT), repeated shrinks -- with
real multi-rank communicators (one thread per rank) over the shared-memory
fake HIP + RCCL (csrc/fakes/fake_hip_rccl.cpp), whose communicators and
streams are heap objects, so any double abort or use after abort is an
ASan report and any unsynchronized hand-off a TSan one.  GPU code is not
involved: the pool has no GPU sanitizer; this is the host half of SURVEY
§5.2."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


SANITIZERS = {
    'asan': ['-fsanitize=address,undefined',
             '-fno-sanitize-recover=undefined'],
    # the abort flag is set from another thread while connect / all-reduce
    # poll it (scenarios 4-5): ThreadSanitizer checks that hand-off
    'tsan': ['-fsanitize=thread'],
}


@pytest.mark.parametrize('sanitizer', sorted(SANITIZERS))
def test_fence_failure_paths_under_sanitizers(tmp_path, sanitizer):
    cxx = shutil.which('g++')
    if cxx is None or not os.path.exists('/opt/rocm/include/rccl/rccl.h'):
        pytest.skip('needs g++ and the ROCm headers')
    san = SANITIZERS[sanitizer] + ['-fno-omit-frame-pointer', '-g', '-O1']
    inc = ['-std=c++17', '-D__HIP_PLATFORM_AMD__', '-I/opt/rocm/include',
           '-I' + os.path.join(ROOT, 'csrc'),
           '-I' + os.path.join(ROOT, 'csrc', 'runtime')]
    fake = str(tmp_path / 'libkiosk_fake_hip_rccl.so')
    native = os.path.join(ROOT, 'tests', 'native')
    subprocess.run([cxx] + san + inc + [
        '-shared', '-fPIC', '-fvisibility=hidden',
        os.path.join(ROOT, 'csrc', 'fakes', 'fake_hip_rccl.cpp'),
        os.path.join(ROOT, 'csrc', 'runtime', 'shmcomm.cpp'), '-o', fake,
        '-pthread'], check=True, timeout=300)
    exe = str(tmp_path / 'fence_asan')
    subprocess.run([cxx] + san + inc + [
        os.path.join(native, 'fence_asan_main.cpp'),
        os.path.join(ROOT, 'csrc', 'runtime', 'fence.cpp'),
        os.path.join(ROOT, 'csrc', 'runtime', 'trace.cpp'),
        fake, '-Wl,-rpath,' + str(tmp_path), '-ldl', '-pthread', '-o', exe],
        check=True, timeout=300)
    env = dict(os.environ, KIOSK_RCCL_LIB=fake, KIOSK_ROCTX='0',
               FAKE_RCCL_DIR=str(tmp_path),
               ASAN_OPTIONS='detect_leaks=1:abort_on_error=0',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1',
               TSAN_OPTIONS='halt_on_error=1:second_deadlock_stack=1')
    proc = subprocess.run([exe], env=env, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=120)
    text = proc.stdout + proc.stderr
    assert proc.returncode == 0, text[-4000:]
    assert 'PASSED: 0 failure(s)' in proc.stdout, text[-4000:]
    assert 'AddressSanitizer' not in text and 'runtime error' not in text
    assert 'ThreadSanitizer' not in text, text[-4000:]
    assert proc.stdout.count('ok ') >= 23
    # every generation's segment was unlinked
    assert not [f for f in os.listdir(str(tmp_path))
                if f.startswith('kiosk-shm-')]
