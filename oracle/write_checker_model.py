"""Python restatement of fdbrpc/AsyncFileWriteChecker.h's checksum history --
TEST INFRASTRUCTURE ONLY (the checker for tests/test_write_checker.py).

Follows the reference line by line: LRU (:107-194), process-wide budget
(:222-227), verifyChecksum (:244-275), updateChecksumHistory (:283-331),
truncate (:76-84), sync (:87-92), destructor (:205-208).  Page checksums come
from the pinned CRC-32C oracle with the checker's seed 0xab12fd93 (:298).
"""
from oracle import oracle as O

PAGE = 4096
SEED = 0xAB12FD93


class Budget:
    value = None  # static Optional<int> checksumHistoryBudget


class LRU:
    def __init__(self):
        self.step = 0
        self.step_to_key = {}
        self.key_to_step = {}
        self.contents = {}

    def update(self, page, info):
        if page in self.key_to_step:
            del self.step_to_key[self.key_to_step[page]]
        self.key_to_step[page] = self.step
        self.step_to_key[self.step] = page
        self.contents[page] = info
        self.step += 1

    def truncate(self, page):
        for k in sorted(k for k in self.key_to_step if k >= page):
            del self.step_to_key[self.key_to_step[k]]
            del self.key_to_step[k]

    def size(self):
        return len(self.key_to_step)

    def exist(self, page):
        return page in self.key_to_step

    def find(self, page):
        return self.contents[page] if page in self.key_to_step else (0, 0)

    def remove(self, page):
        if page not in self.key_to_step:
            return
        self.contents.pop(page, None)
        del self.step_to_key[self.key_to_step[page]]
        del self.key_to_step[page]


class WriteCheckerModel:
    def __init__(self, budget):
        if Budget.value is None:
            Budget.value = budget
        self.lru = LRU()
        self.writing = set()
        self.synced = 0
        self.succeed = 0
        self.failed = 0

    def close(self):
        Budget.value += self.lru.size()

    def _update(self, update, offset, length, buf, now_ms=0):
        pages = []
        fails = 0
        page = offset // PAGE + 1
        slack = offset % PAGE
        start = 0
        if slack:
            page += 1
            start += PAGE - slack
        page_end = (offset + length) // PAGE
        while page < page_end:
            checksum = O.crc32c(SEED, bytes(buf[start:start + PAGE]))
            if update:
                self.writing.add(page)
                pages.append(page)
                if not self.lru.exist(page):
                    if Budget.value > 0:
                        Budget.value -= 1
                    else:
                        break
                self.lru.update(page, (checksum, now_ms))
            else:
                if not self._verify(page, checksum):
                    break
                if self._last_failed:
                    fails += 1
            start += PAGE
            page += 1
        return pages, fails

    def _verify(self, page, checksum):
        self._last_failed = False
        if not self.lru.exist(page):
            return True
        cs, ts = self.lru.find(page)
        if ts < self.synced:
            if cs != checksum:
                self.failed += 1
                self._last_failed = True
            else:
                Budget.value += 1
                self.lru.remove(page)
                self.succeed += 1
            return True
        return False

    def write(self, buf, offset, now_ms):
        return self._update(True, offset, len(buf), buf, now_ms)[0]

    def write_done(self, pages):
        for p in pages:
            self.writing.discard(p)

    def read(self, buf, offset):
        return self._update(False, offset, len(buf), buf)[1]

    def sync(self, now_ms):
        self.synced = now_ms

    def truncate(self, size):
        old = self.lru.size()
        self.lru.truncate(size // PAGE)
        Budget.value += old - self.lru.size()

    def history(self):
        return {p: self.lru.find(p) for p in self.lru.key_to_step}

    def sweep_pages(self, cap):
        """Pages the sweep actor (AsyncFileWriteChecker.h:218-232) visits next:
        from the least recently used on (leastRecentlyUsedPage, :168-173),
        stopping where it would wait for a page being written."""
        out = []
        for step in sorted(self.lru.step_to_key):
            p = self.lru.step_to_key[step]
            if p in self.writing or len(out) == cap:
                break
            out.append(p)
        return out
