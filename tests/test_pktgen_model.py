"""CPU checks of the generator test cases (tests/pktgen_templates.py): each case table must
rebuild its template from the template's own field values, and the oracle's clone +
set_bit_range + checksum refresh (what the GPU generator is compared with) must equal the
builder called with each packet's arguments.  No GPU: this pins the expectations the -m gpu
generator tests rely on."""
import numpy as np
import pytest

import oracle
from pktgpu import gen, pktgen

import pktgen_templates as T


@pytest.mark.parametrize("name", gen.REFERENCE_22_NAMES)
def test_case_table_rebuilds_template(name):
    tpl = T.template_bytes(name)
    fields, csum, build = T.TEMPLATES[name]
    n = 1
    slab = np.frombuffer(tpl, np.uint8).copy()
    chain = oracle.parse_batch(slab, 1, stride=len(tpl), columns=["status", "n_hdrs", "hdr_type", "hdr_off"])
    assert chain["status"][0] == 0
    specs = []
    for arg, hdr, fld, occ, _hi in fields:
        f = pktgen.Field(hdr, fld, occ)
        specs.append((f.hdr, f.occurrence, f.start, f.end))
    vals, found = oracle.extract_fields(slab, n, chain, specs, stride=len(tpl))
    assert all(int(x[0]) for x in found), name
    v = {arg: int(vals[j][0]) for j, (arg, *_r) in enumerate(fields)}
    assert build(v).to_vec() == tpl


@pytest.mark.parametrize("name", gen.REFERENCE_22_NAMES)
def test_oracle_generation_equals_builder(name):
    tpl = T.template_bytes(name)
    n, first = 64, 77
    gf, values, host_vals, csum, build = T.make_case(name, n, first)
    stride = ((len(tpl) + 15) & ~15) + 16
    want = T.oracle_batch(tpl, n, stride, [(f.hdr, f.occurrence, f.start, f.end) for f in gf], host_vals, csum)
    for i in range(n):
        assert want[i, :len(tpl)].tobytes() == build(T.builder_args(name, host_vals, i)).to_vec(), (name, i)


def test_value_kinds():
    g = np.arange(5, 10, dtype=np.uint64)
    assert list(pktgen.Field("Ether", "etype", kind="inc", base=3, step=2, count=3).value(g)) == \
        [3 + 2 * (k % 3) for k in range(5, 10)]
    assert list(pktgen.Field("Ether", "etype", kind="inc", base=0xFFFF, step=1).value(g)) == \
        [(0xFFFF + k) & 0xFFFF for k in range(5, 10)]
    # splitmix64 reference values (seed 0: the published first outputs of the generator)
    assert int(pktgen.splitmix64(np.uint64(0))) == 0xE220A8397B1DCDAF
    r = pktgen.Field("IPv4", "src", kind="random", base=0).value(np.array([0], np.uint64))
    assert int(r[0]) == 0xE220A8397B1DCDAF & 0xFFFFFFFF
