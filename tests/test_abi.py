"""C-ABI checks that need no GPU: the library loads, exports every function
include/srtp_mi355x.h declares, and its struct layouts / enum values match
the reference header (include/srtp.h) they claim to replace."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

import libsrtp_amd as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "srtp_mi355x.h")
REF_INC = "/root/reference/include"


def declared_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", text)
    names = set()
    # a name followed by "(" -- but not "(*": a function-pointer typedef
    for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\((?!\s*\*)", text):
        name = m.group(1)
        if name.startswith("srtp_") and not name.endswith("_func_t"):
            names.add(name)
    return sorted(names)


def test_every_declared_symbol_is_exported():
    lib = C.CDLL(L.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert declared_functions(), "header parse found nothing"
    assert not missing, missing


def test_status_values_match_reference_header():
    assert L.Status.auth_fail == 7 and L.Status.replay_fail == 9
    assert L.Status.buffer_small == 28 and L.Status.cryptex_err == 29


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include HEADER
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n",
    sizeof(srtp_policy_t), offsetof(srtp_policy_t, rtp),
    offsetof(srtp_policy_t, key), offsetof(srtp_policy_t, keys),
    offsetof(srtp_policy_t, use_mki), offsetof(srtp_policy_t, window_size),
    offsetof(srtp_policy_t, allow_repeat_tx),
    offsetof(srtp_policy_t, use_cryptex), offsetof(srtp_policy_t, next),
    sizeof(srtp_crypto_policy_t));
  printf("%d %d %d %d %d\n", (int)srtp_err_status_bad_mki,
    (int)srtp_err_status_pkt_idx_adv, (int)ssrc_any_outbound,
    (int)event_packet_index_limit, (int)srtp_profile_aead_aes_256_gcm);
  return 0;
}
"""


def _layout(header, inc):
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "l.c")
        exe = os.path.join(d, "l")
        open(src, "w").write(LAYOUT_C.replace("HEADER", '"%s"' % header))
        subprocess.check_call(["gcc", "-I", inc, src, "-o", exe])
        return subprocess.check_output([exe]).decode()


@pytest.mark.skipif(not os.path.isdir(REF_INC),
                    reason="reference headers only in the build container")
def test_struct_layout_matches_reference():
    ours = _layout(HDR, os.path.dirname(HDR))
    ref = _layout(os.path.join(REF_INC, "srtp.h"), REF_INC)
    assert ours == ref


def test_ctypes_policy_matches_c_layout():
    out = _layout(HDR, os.path.dirname(HDR)).split()
    assert int(out[0]) == C.sizeof(L.Policy)
    assert int(out[9]) == C.sizeof(L.CryptoPolicy)


def test_no_gpu_fails_loudly():
    lib = L.lib()
    if lib.srtp_mi355x_gpu_available():
        pytest.skip("GPU present")
    assert lib.srtp_init() == L.Status.init_fail
    h = C.c_void_p()
    p = L.Policy()
    assert lib.srtp_create(C.byref(h), None) == L.Status.init_fail
