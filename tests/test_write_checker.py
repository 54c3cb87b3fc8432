"""The batched lost-write checker (include/fdb_writechecker.h) against a line-by-line
restatement of fdbrpc/AsyncFileWriteChecker.h (oracle/write_checker_model.py),
replaying random I/O streams: writes of any size and alignment, reads of good
and lost-write data, syncs, truncates, an exhausted history budget."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import write_checker_model as M

FILE_PAGES = 96


def scenario(seed, nops=400, budget=200):
    """Yields (op, args) with file contents evolving like a real file."""
    rng = np.random.default_rng(seed)
    disk = np.zeros(FILE_PAGES * 4096, np.uint8)
    t = 1
    ops = []
    for _ in range(nops):
        t += int(rng.integers(1, 5))
        r = rng.random()
        off = int(rng.integers(0, FILE_PAGES * 4096 - 1))
        ln = int(min(rng.choice([100, 4096, 8192, 3 * 4096 + 17, 40000, 200000]), disk.size - off))
        if rng.random() < 0.3:  # page-aligned I/O
            off = off // 4096 * 4096
            ln = min(ln // 4096 * 4096 or 4096, disk.size - off)
        if r < 0.4:
            data = rng.integers(0, 256, ln, dtype=np.uint8)
            disk[off:off + ln] = data
            ops.append(("write", data.copy(), off, t))
        elif r < 0.75:
            data = disk[off:off + ln].copy()
            if rng.random() < 0.2 and ln:  # a lost write / bit rot seen by the read
                data[int(rng.integers(0, ln))] ^= 0x40
            ops.append(("read", data, off, t))
        elif r < 0.9:
            ops.append(("sync", None, 0, t))
        else:
            ops.append(("truncate", None, int(rng.integers(0, disk.size)), t))
    return ops, budget


def replay(ops, budget, native_factory):
    M.Budget.value = None
    model = M.WriteCheckerModel(budget)
    nat = native_factory(budget)
    for op, data, off, t in ops:
        if op == "write":
            pm = model.write(data, off, t)
            pn = nat.write(data, off, t)
            assert pm == pn
            model.write_done(pm)
            nat.write_done(pn)
        elif op == "read":
            assert model.read(data, off) == nat.read(data, off)
        elif op == "sync":
            model.sync(t)
            nat.sync(t)
        else:
            model.truncate(off)
            nat.truncate(off)
        st = nat.stats()
        assert (st["succeed"], st["fail"], st["history"]) == (model.succeed, model.failed, model.lru.size())
        assert nat.sweep_pages(37) == model.sweep_pages(37)
    hist = model.history()
    for p in range(1, FILE_PAGES + 2):
        assert nat.history_entry(p) == (hist.get(p))
    return model, nat


def test_checker_matches_reference_model_host():
    import foundationdb_amd.write_checker as W
    for seed, budget in ((1, 200), (2, 12), (3, 100000)):
        ops, _ = scenario(seed, budget=budget)
        W.reset_budget()
        model, nat = replay(ops, budget, lambda b: W.WriteChecker(b, gpu_threshold=0))
        assert W.budget() == M.Budget.value
        nat.close()
        model.close()
        assert W.budget() == M.Budget.value


def test_reference_quirks_kept():
    """Single aligned 4 KiB writes are not recorded (updateChecksumHistory's
    pageEnd excludes the last full page); truncate(size) also drops page size/4096."""
    import foundationdb_amd.write_checker as W
    W.reset_budget()
    c = W.WriteChecker(100, gpu_threshold=0)
    assert c.write(np.ones(4096, np.uint8), 0, 5) == []
    assert c.write(np.ones(3 * 4096, np.uint8), 4096, 5) == [2, 3]
    c.truncate(3 * 4096)
    assert c.stats()["history"] == 1 and c.history_entry(2) is not None
    c.close()


def test_sweep_order_and_batched_verification():
    """fdb_wc_sweep_pages lists history pages from the least recently used on
    and stops at a page being written (where the reference's sweep actor
    waits); reading the listed pages' bytes verifies them in one batch: synced
    pages that match leave the history, a lost write is reported.  The
    reference's own sweep reads offset page*4096, whose 4096 bytes hold no
    full page by updateChecksumHistory's rule: it verifies nothing."""
    import foundationdb_amd.write_checker as W
    W.reset_budget()
    c = W.WriteChecker(1000, gpu_threshold=0)
    rng = np.random.default_rng(4)
    data = rng.integers(0, 256, 64 * 4096, dtype=np.uint8)
    pages = c.write(data[:20 * 4096], 0, 10)  # pages 1..19 (the last full page is left out)
    c.write_done(pages)
    late = c.write(data[30 * 4096:34 * 4096], 30 * 4096, 11)  # pages 31..33, still being written
    assert c.sweep_pages(100) == list(range(1, 20))
    assert c.sweep_pages(5) == [1, 2, 3, 4, 5]
    c.write_done(late)
    assert c.sweep_pages(100) == list(range(1, 20)) + late
    c.sync(12)
    # the reference's sweep read for page 1: offset 4096, 4096 bytes -> no full page checked
    assert c.read(data[4096:8192], 4096) == 0 and c.stats()["history"] == 22
    # the batched sweep: bytes [(p-1)*4096, p*4096) of pages 1..19 in one read, page 7 lost
    disk = data[:20 * 4096].copy()
    disk[6 * 4096 + 100] ^= 1
    failures = c.read(disk, 0)
    assert failures == 1
    st = c.stats()
    assert st["fail"] == 1 and st["succeed"] == 18
    assert c.sweep_pages(100)[0] == 7  # the lost write stays in the history
    c.close()


class _LRU2:
    """The reference test's second LRU (fdbrpc/AsyncFileWriteChecker.cpp:31-161):
    most recent at the head, truncate(n) drops pages [n, maxFullPagePlusOne)."""

    def __init__(self):
        from collections import OrderedDict
        self.m = OrderedDict()  # least recently used first
        self.max_plus_one = 0

    def update(self, page, info):
        self.m.pop(page, None)
        self.m[page] = info
        self.max_plus_one = max(self.max_plus_one, page + 1)

    def remove(self, page):
        self.m.pop(page, None)

    def truncate(self, n):
        for i in range(n, self.max_plus_one):
            self.remove(i)
        self.max_plus_one = min(self.max_plus_one, n)

    def least_recently_used(self):
        return next(iter(self.m)) if self.m else 0


def test_reference_lru_sequence():
    """The reference's own LRU test (/fdbrpc/AsyncFileWriteChecker/LRU,
    fdbrpc/AsyncFileWriteChecker.cpp:164-229) replayed through the checker's
    C ABI and the line-by-line model: 1000 steps, each an update (p > 0.5 or
    empty history), a removal (p < 0.45) or a truncate, pages in [1, 1000).
    update(page, info) is a write of 8192 bytes at (page - 1) * 4096 (it
    records exactly that page: updateChecksumHistory's pageEnd leaves out the
    last full page), with fresh random bytes so the checksum changes each
    time; remove(page) is a sync followed by a read of the page's bytes (a
    synced page that verifies leaves the history, verifyChecksum :244-275);
    truncate(page) is truncate(page * 4096) (maxFullPage = size / 4096,
    :76-84).  After every step: existence and (checksum, timestamp) of the
    pages touched, and the least recently used page (fdb_wc_sweep_pages) with
    its entry, as the reference compares them against LRU2."""
    import foundationdb_amd.write_checker as W
    rng = np.random.default_rng(20240518)
    W.reset_budget()
    M.Budget.value = None
    nat = W.WriteChecker(1 << 20, gpu_threshold=0)
    model = M.WriteCheckerModel(1 << 20)
    lru2 = _LRU2()
    content = {}  # the bytes each recorded page holds on "disk"
    limit, t = 1000, 1
    for _ in range(1000):
        t += 1
        r = rng.random()
        if not lru2.m or r > 0.5:  # add / update
            page = int(rng.integers(1, limit))
            if page in lru2.m:
                assert nat.history_entry(page) == lru2.m[page]
            data = rng.integers(0, 256, 8192, dtype=np.uint8)
            off = (page - 1) * 4096
            assert nat.write(data, off, t) == [page]
            nat.write_done([page])
            model.write_done(model.write(data, off, t))
            content[page] = data
            lru2.update(page, (O.crc32c(M.SEED, data[:4096].tobytes()), t))
            assert nat.history_entry(page) == lru2.m[page] == model.history()[page]
        elif r < 0.45:  # remove
            page = list(lru2.m)[int(rng.integers(0, len(lru2.m)))]
            assert nat.history_entry(page) == lru2.m[page]
            nat.sync(t)
            model.sync(t)
            t += 1
            assert nat.read(content[page], (page - 1) * 4096) == 0
            model.read(content[page], (page - 1) * 4096)
            lru2.remove(page)
            assert nat.history_entry(page) is None and page not in model.history()
        else:  # truncate
            keys = list(lru2.m)
            page, page2 = (keys[int(rng.integers(0, len(keys)))] for _ in range(2))
            nat.truncate(page * 4096)
            model.truncate(page * 4096)
            lru2.truncate(page)
            if page2 >= page:
                assert nat.history_entry(page2) is None and page2 not in lru2.m
        assert nat.stats()["history"] == len(lru2.m) == model.lru.size()
        if lru2.m:
            lru_page = lru2.least_recently_used()
            assert nat.sweep_pages(1) == [lru_page] == model.sweep_pages(1)
            assert nat.history_entry(lru_page) == lru2.m[lru_page]
    nat.close()
    model.close()


@pytest.mark.gpu
def test_checker_gpu_pipeline_and_device_batches(cuda):
    import torch
    import foundationdb_amd.write_checker as W
    ops, budget = scenario(7, nops=300, budget=150)
    # host buffers through the pinned GPU pipeline (threshold 1 page)
    W.reset_budget()
    model, nat = replay(ops, budget, lambda b: W.WriteChecker(b, gpu_threshold=1))
    nat.close()
    # device-resident buffers, asynchronous submit + poll/wait
    W.reset_budget()
    M.Budget.value = None
    model = M.WriteCheckerModel(budget)
    nat = W.WriteChecker(budget, gpu_threshold=0)
    last = 0
    keep = []  # device buffers stay alive until their tickets are applied
    for op, data, off, t in ops:
        if op in ("write", "read"):
            d = torch.from_numpy(data).to(cuda)
            torch.cuda.synchronize()  # the data is on the device before the checker's stream reads it
            keep.append(d)
        if op == "write":
            model.write_done(model.write(data, off, t))
            last = nat.write_device(d, off, t)
            nat.poll()
        elif op == "read":
            model.read(data, off)
            last = nat.read_device(d, off)
        elif op == "sync":
            model.sync(t)
            nat.sync(t)  # drains the queue first: submission order is kept
        else:
            model.truncate(off)
            nat.truncate(off)
    nat.wait(last)
    st = nat.stats()
    assert (st["succeed"], st["fail"], st["history"]) == (model.succeed, model.failed, model.lru.size())
    hist = model.history()
    for p in range(1, FILE_PAGES + 2):
        assert nat.history_entry(p) == hist.get(p)
    nat.close()
