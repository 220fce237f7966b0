import pytest
pytestmark = pytest.mark.gpu


def test_convert_v1_to_v2_device(oracle):
    """yconvert_updates_v1_to_v2_batch_device == Update::decode_v1(u).encode_v2() per update."""
    import ymerge
    import workloads
    b = workloads.text_docs(20, 100, seed=77, max_clients=3)
    e = ymerge.Engine(0)
    out, off, st = e.convert_v1_to_v2_host(b.data, b.upd_off)
    e.close()
    assert not st.any()
    for i in range(b.n_updates):
        u = bytes(b.data[int(b.upd_off[i]):int(b.upd_off[i + 1])])
        assert out[int(off[i]):int(off[i + 1])].tobytes() == oracle.convert_update_v1_to_v2(u), i
