"""Host-code sanitizers (race detection / sanitizers):
the native pair collator (csrc/host/collate.cpp) built with
AddressSanitizer + UndefinedBehaviorSanitizer and driven over random graph
stores and batches with exactly sized buffers (tests/native/asan_collate.cpp,
tools/asan_host.sh).  GPU sanitizers are not available on this pool; the HIP
kernels are covered by the determinism / oracle-parity tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_available():
    if shutil.which('g++') is None:
        return False
    probe = subprocess.run(['g++', '-fsanitize=address', '-x', 'c++', '-',
                            '-o', os.devnull], input=b'int main(){}',
                           capture_output=True)
    return probe.returncode == 0


@pytest.mark.skipif(not _asan_available(), reason='no g++ with ASan')
def test_native_collator_under_asan_ubsan(tmp_path):
    res = subprocess.run(['bash', os.path.join(ROOT, 'tools', 'asan_host.sh'),
                          str(tmp_path)], capture_output=True, text=True,
                         timeout=1200)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert 'asan_collate: ok' in out
    assert 'ERROR: AddressSanitizer' not in out
    assert 'runtime error' not in out        # UBSan report
