"""Native TCPStore append: the append is one server-side command, so concurrent appends of
IDENTICAL bytes from many clients all land — the old client-side read / compare_set loop lost one of two equal
appends (it took 'returned value == new' as success)."""
import threading

from paddle2_amd.distributed.store import TCPStore, TorchStore, _LIVE, release_clones


def test_concurrent_identical_appends_all_land():
    master = TCPStore("127.0.0.1", 0, True, 1, 30)
    clients = [TorchStore(TCPStore("127.0.0.1", master.port, False, 1, 30)) for _ in range(8)]
    n = 50

    def work(c):
        for _ in range(n):
            c.append("k", b"x")

    ts = [threading.Thread(target=work, args=(c,)) for c in clients]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert bytes(master.get("k")) == b"x" * (8 * n)
    master.shutdown()


def test_clones_released_after_destroy():
    master = TCPStore("127.0.0.1", 0, True, 1, 30)
    root = TorchStore(master)
    c = root.clone()
    c.set("a", b"1")
    assert bytes(root.get("a")) == b"1"
    assert any(s is c for s in _LIVE)
    release_clones()
    assert not any(s is c for s in _LIVE) and any(s is root for s in _LIVE)
    master.shutdown()
