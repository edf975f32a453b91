"""GPU packet generation (pktgpu.pktgen) against the host builders and the oracle."""
import numpy as np
import pytest

import oracle
from pktgpu import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible")
    import pktgpu
    return pktgpu.Parser(0)


def test_broadcast_clones_template(P):
    import torch
    from pktgpu import pktgen
    tpl = pktgen.udp_template()
    src = torch.from_numpy(np.frombuffer(tpl, np.uint8).copy()).cuda()
    out = P.broadcast(src, 1000, 80).cpu().numpy().reshape(1000, 80)
    want = np.zeros(80, np.uint8)
    want[:len(tpl)] = np.frombuffer(tpl, np.uint8)
    assert (out == want).all()


def test_gen_udp_matches_host_builder(P):
    """Every packet equals create_udp_packet(...) with that packet's field values."""
    import torch
    from pktgpu import pktgen
    n = 20000
    rng = np.random.default_rng(12)
    f = {"eth_dst": rng.integers(0, 2**48, n, dtype=np.uint64),
         "eth_src": rng.integers(0, 2**48, n, dtype=np.uint64),
         "ipv4_diffserv": rng.integers(0, 256, n).astype(np.uint64),
         "ipv4_identification": rng.integers(0, 65536, n).astype(np.uint64),
         "ipv4_ttl": rng.integers(1, 256, n).astype(np.uint64),
         "ipv4_src": rng.integers(0, 2**32, n, dtype=np.uint64),
         "ipv4_dst": rng.integers(0, 2**32, n, dtype=np.uint64),
         "udp_src": rng.integers(0, 65536, n).astype(np.uint64),
         "udp_dst": rng.integers(0, 65536, n).astype(np.uint64)}
    slab = pktgen.gen_udp(P, n, {k: torch.from_numpy(v).cuda() for k, v in f.items()})
    got = slab.cpu().numpy().reshape(n, 64)
    for i in list(range(0, n, 997)) + [n - 1]:
        mac = lambda x: ":".join(f"{(int(x) >> (40 - 8 * k)) & 0xFF:02x}" for k in range(6))  # noqa: E731
        ip = lambda x: ".".join(str((int(x) >> (24 - 8 * k)) & 0xFF) for k in range(4))  # noqa: E731
        want = gen.create_udp_packet(mac(f["eth_dst"][i]), mac(f["eth_src"][i]), False, 10, 3, 5,
                                     ip(f["ipv4_src"][i]), ip(f["ipv4_dst"][i]), int(f["ipv4_diffserv"][i]),
                                     int(f["ipv4_ttl"][i]), int(f["ipv4_identification"][i]), 0x4000, [],
                                     int(f["udp_dst"][i]), int(f["udp_src"][i]), False, bytes(range(22))).to_vec()
        assert got[i].tobytes() == want, i
    # and the whole slab parses with valid checksums (oracle)
    r = oracle.parse_batch(got, n, stride=64)
    assert (r["status"] == 0).all()
    assert np.array_equal(r["ipv4_header_checksum"], r["ipv4_csum_calc"])
    assert np.array_equal(r["udp_dst"], f["udp_dst"].astype(np.uint16))
