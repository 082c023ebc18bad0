"""paddle.reader — legacy reader decorators (reference: python/paddle/reader/decorator.py).

A *reader* is a zero-argument callable returning an iterable of samples; the decorators compose them:
``cache``, ``map_readers``, ``shuffle`` (buffered), ``chain``, ``compose`` (zip, optionally checking alignment),
``buffered`` (a producer thread ahead of the consumer), ``firstn``, ``xmap_readers`` (thread pool map, ordered or
not) and ``multiprocess_reader`` (one process per reader feeding a queue).
"""
from __future__ import annotations

import itertools
import multiprocessing
import queue
import random
import threading

__all__ = ["cache", "map_readers", "shuffle", "chain", "compose", "ComposeNotAligned", "buffered", "firstn",
           "xmap_readers", "multiprocess_reader"]


def cache(reader):
    data = list(reader())

    def r():
        yield from data

    return r


def map_readers(func, *readers):
    def r():
        for items in zip(*[rd() for rd in readers]):
            yield func(*items)

    return r


def shuffle(reader, buf_size):
    def r():
        buf = []
        for s in reader():
            buf.append(s)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        if buf:
            random.shuffle(buf)
            yield from buf

    return r


def chain(*readers):
    def r():
        yield from itertools.chain(*[rd() for rd in readers])

    return r


class ComposeNotAligned(ValueError):
    pass


def compose(*readers, **kwargs):
    check_alignment = kwargs.pop("check_alignment", True)

    def flat(x):
        return x if isinstance(x, tuple) else (x,)

    def r():
        its = [rd() for rd in readers]
        if not check_alignment:
            for outs in zip(*its):
                yield sum((flat(o) for o in outs), ())
            return
        for outs in itertools.zip_longest(*its):
            if any(o is None for o in outs):
                raise ComposeNotAligned("outputs of readers are not aligned")
            yield sum((flat(o) for o in outs), ())

    return r


class _End:
    pass


def buffered(reader, size):
    def r():
        q = queue.Queue(maxsize=size)

        def fill():
            for s in reader():
                q.put(s)
            q.put(_End)

        t = threading.Thread(target=fill, daemon=True)
        t.start()
        while True:
            s = q.get()
            if s is _End:
                break
            yield s
        t.join()

    return r


def firstn(reader, n):
    def r():
        yield from itertools.islice(reader(), n)

    return r


class XmapEndSignal:
    pass


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    """Map ``reader``'s samples through ``mapper`` on ``process_num`` threads (in order when ``order``)."""
    def r():
        inq, outq = queue.Queue(buffer_size), queue.Queue(buffer_size)

        def feed():
            for i, s in enumerate(reader()):
                inq.put((i, s))
            for _ in range(process_num):
                inq.put(XmapEndSignal)

        def work():
            while True:
                item = inq.get()
                if item is XmapEndSignal:
                    outq.put(XmapEndSignal)
                    return
                i, s = item
                outq.put((i, mapper(s)))

        threads = [threading.Thread(target=feed, daemon=True)] + [
            threading.Thread(target=work, daemon=True) for _ in range(process_num)]
        for t in threads:
            t.start()
        done, nxt, pending = 0, 0, {}
        while done < process_num:
            item = outq.get()
            if item is XmapEndSignal:
                done += 1
                continue
            if not order:
                yield item[1]
                continue
            pending[item[0]] = item[1]
            while nxt in pending:
                yield pending.pop(nxt)
                nxt += 1
        while order and nxt in pending:
            yield pending.pop(nxt)
            nxt += 1

    return r


def _mp_worker(reader, q):
    for s in reader():
        q.put(s)
    q.put(None)


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    """One process per reader feeding a shared queue (samples must be picklable)."""
    def r():
        ctx = multiprocessing.get_context("fork")
        q = ctx.Queue(queue_size)
        procs = [ctx.Process(target=_mp_worker, args=(rd, q), daemon=True) for rd in readers]
        for p in procs:
            p.start()
        finished = 0
        while finished < len(readers):
            s = q.get()
            if s is None:
                finished += 1
                continue
            yield s
        for p in procs:
            p.join()

    return r
