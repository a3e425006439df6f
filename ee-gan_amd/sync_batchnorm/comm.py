"""Host-side master/slave rendezvous names of the reference
(sync_batchnorm/comm.py:18-137), kept so code importing them still runs.

The reference's SyncBatchNorm exchanges statistics between replica THREADS
of one process: every slave posts its message to the master, the master's
callback reduces them and hands each replica its reply.  This package runs
one process per GPU instead -- the statistics go over RCCL (or the peer-write
kernel, eegan_hip.peer) inside eegan_hip.functional -- so nothing here is on
the data path.  The classes still behave as documented for in-process use:

  * FutureResult: one-slot handoff, get() blocks until put();
  * SlavePipe(identifier, queue, result).run_slave(msg): post (id, msg), wait
    for the reply, then acknowledge;
  * SyncMaster(callback).register_slave(id) -> SlavePipe;
    run_master(msg): collect [(0, msg), (id, msg_id), ...], call the callback,
    deliver every (id, reply) to its slave, wait for the acknowledgements and
    return the master's own reply.
"""
import collections
import queue
import threading

__all__ = ['FutureResult', 'SlavePipe', 'SyncMaster']


class FutureResult(object):
    """Single-value handoff between two threads (one producer, one consumer)."""

    _EMPTY = object()

    def __init__(self):
        self._value = self._EMPTY
        self._ready = threading.Condition()

    def put(self, result):
        with self._ready:
            if self._value is not self._EMPTY:
                raise AssertionError('FutureResult: previous result not fetched yet')
            self._value = result
            self._ready.notify()

    def get(self):
        with self._ready:
            self._ready.wait_for(lambda: self._value is not self._EMPTY)
            value, self._value = self._value, self._EMPTY
            return value


class SlavePipe(collections.namedtuple('_SlavePipe', ['identifier', 'queue', 'result'])):
    """A slave's end of the rendezvous."""

    def run_slave(self, msg):
        self.queue.put((self.identifier, msg))
        reply = self.result.get()
        self.queue.put(True)   # acknowledgement: the master may start the next round
        return reply


class SyncMaster(object):
    """The master's end: gathers one message per registered slave per round."""

    def __init__(self, master_callback):
        self._master_callback = master_callback
        self._queue = queue.Queue()
        self._slaves = collections.OrderedDict()   # identifier -> FutureResult
        self._in_round = False

    def __getstate__(self):
        return {'master_callback': self._master_callback}

    def __setstate__(self, state):
        self.__init__(state['master_callback'])

    def register_slave(self, identifier):
        if self._in_round:   # a new replication: forget the previous slaves
            if not self._queue.empty():
                raise AssertionError('SyncMaster: messages left over from the previous round')
            self._in_round = False
            self._slaves.clear()
        fut = FutureResult()
        self._slaves[identifier] = fut
        return SlavePipe(identifier, self._queue, fut)

    def run_master(self, master_msg):
        self._in_round = True
        msgs = [(0, master_msg)] + [self._queue.get() for _ in self._slaves]
        replies = self._master_callback(msgs)
        if replies[0][0] != 0:
            raise AssertionError('SyncMaster: the first reply must be the master\'s')
        for ident, reply in replies[1:]:
            self._slaves[ident].put(reply)
        for _ in self._slaves:
            if self._queue.get() is not True:
                raise AssertionError('SyncMaster: expected a slave acknowledgement')
        return replies[0][1]

    @property
    def nr_slaves(self):
        return len(self._slaves)
