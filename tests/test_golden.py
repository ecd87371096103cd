"""Committed golden fixtures (tests/golden/icrc_golden.npz, made by make_golden.py with Python
zlib) against the oracle (CPU), the emulated kernel algorithm (CPU) and the GPU engine."""
import os

import numpy as np
import pytest

import oracle
import kernel_emu

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "icrc_golden.npz"), allow_pickle=False)


def packets(buf):
    for o, L in zip(G["off"], G["lens"]):
        yield buf[int(o): int(o) + int(L)]


def test_fixture_shape():
    assert G["lens"].size >= 80
    assert {"kat", "raw"} <= set(G["kinds"].tolist())


def test_oracle_matches_golden():
    got = oracle.compute_icrc_batch(G["buf"], G["off"], G["lens"])
    np.testing.assert_array_equal(got, G["icrc"])


def test_oracle_verify_matches_golden():
    vb = G["verify_buf"].copy()
    ok = [oracle.is_icrc_valid(np.ascontiguousarray(p)) for p in packets(vb)]
    np.testing.assert_array_equal(np.array(ok, np.uint8), G["verify_ok"])


def test_kernel_emulation_matches_golden():
    import icrc_amd

    img = icrc_amd.table_image()
    for i, p in enumerate(packets(G["buf"])):
        if i % 3 == 0 or p.size < 600:  # keep the pure-python emulation quick
            assert kernel_emu.icrc(img, np.ascontiguousarray(p)) == int(G["icrc"][i])


@pytest.mark.gpu
def test_gpu_matches_golden(engine):
    import torch

    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    n = G["lens"].size
    d_buf, d_off, d_len = d(G["buf"]), d(G["off"]), d(G["lens"])
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(), stream=s)
    d_vbuf = d(G["verify_buf"])
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_vbuf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(), stream=s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), G["icrc"])
    np.testing.assert_array_equal(d_ok.cpu().numpy(), G["verify_ok"])


def test_oracle_rx_parse_pinned_by_reference_test_packet():
    """The oracle's to_rdma_message restatement decodes the four header shapes of the reference's
    rust_driver/src/device/software/tests/test_packet.rs:16-185 to the values those tests assert."""
    import rx_cases

    for name, pkt, expect in rx_cases.reference_cases():
        d = oracle.rx_parse(pkt.copy(), [0], [pkt.size])[0]
        rx_cases.check_reference_expect(d, expect, name)
