"""CPU tier: the `mirroritems` sub-bench's workload (bench.mirror_items_workload)
-- item columns shaped as vc_mirror_items, every level present, and the
bit-set path run on the host (tests/native imgcheck) equal to the oracle
batch form the bench times as its CPU leg."""
import numpy as np

import bench as B
import imgcheck_ffi as I
import oracle_ffi as O
from vproxy_amd.mirror import MirrorFilters, items_struct


def test_mirror_items_workload_on_host():
    box = {}

    def mf_of(filters):
        mf = MirrorFilters()
        box["arr"], box["n"] = mf.build(filters)
        return mf
    filters, mf, tcols, dcols, idx = B.mirror_items_workload(20000, "cpu", mf_of)
    n = len(idx)
    cols = {k: v.numpy() for k, v in dcols.items()}
    assert cols["mac_src"].shape == (6 * n,) and cols["ip_src"].shape == (n, 16)
    lens = cols["ip_src_len"]
    assert set(np.unique(lens)) == {0, 4, 16}
    assert (cols["transport"] == -1).mean() > 0.1 and (cols["app"] != -1).mean() > 0.1
    ids = {}
    oarr = O.mirror_filters(filters, ids)
    assert ids == mf.ids
    oid = mf.id_of("tcp-lb", create=False)
    want = O.mirror_match_batch_np(oarr, len(filters), oid, cols, nthreads=4)
    got = I.mirror_sw(box["arr"], box["n"], oid, items_struct(cols), n)
    np.testing.assert_array_equal(got, want)
    assert (want != 0).mean() > 0.2
