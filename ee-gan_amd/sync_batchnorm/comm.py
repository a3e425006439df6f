"""Host-side master/slave rendezvous (API of sync_batchnorm/comm.py:18-137).

Not used by the MI355X path -- statistics travel over RCCL between ranks,
never through host threads -- but kept so code importing these names runs."""
import collections
import queue
import threading

__all__ = ['FutureResult', 'SlavePipe', 'SyncMaster']


class FutureResult(object):
    def __init__(self):
        self._result = None
        self._cond = threading.Condition(threading.Lock())

    def put(self, result):
        with self._cond:
            assert self._result is None, 'Previous result has not been fetched.'
            self._result = result
            self._cond.notify()

    def get(self):
        with self._cond:
            while self._result is None:
                self._cond.wait()
            r, self._result = self._result, None
            return r


class SlavePipe(collections.namedtuple('_SlavePipeBase', ['identifier', 'queue', 'result'])):
    def run_slave(self, msg):
        self.queue.put((self.identifier, msg))
        ret = self.result.get()
        self.queue.put(True)
        return ret


class SyncMaster(object):
    def __init__(self, master_callback):
        self._master_callback = master_callback
        self._queue = queue.Queue()
        self._registry = collections.OrderedDict()
        self._activated = False

    def register_slave(self, identifier):
        if self._activated:
            assert self._queue.empty(), 'Queue is not clean before next initialization.'
            self._activated = False
            self._registry.clear()
        future = FutureResult()
        self._registry[identifier] = future
        return SlavePipe(identifier, self._queue, future)

    def run_master(self, master_msg):
        self._activated = True
        msgs = [(0, master_msg)] + [self._queue.get() for _ in range(self.nr_slaves)]
        results = self._master_callback(msgs)
        assert results[0][0] == 0, 'The first result should belong to the master.'
        for i, res in results[1:]:
            self._registry[i].put(res)
        for _ in range(self.nr_slaves):
            assert self._queue.get() is True
        return results[0][1]

    @property
    def nr_slaves(self):
        return len(self._registry)
