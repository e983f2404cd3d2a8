"""Per-sample audio streaming out of generate() (reference:
vibevoice/modular/streamer.py:13-264; used by generate() at
modeling_vibevoice_inference.py:443-447, 540-553, 663-665 and by
demo/gradio_demo.py's streaming player).

Same classes, argument meaning and queue protocol as the reference:

* `AudioStreamer(batch_size, stop_signal=None, timeout=None)`: one FIFO per
  sample.  `put(audio_chunks, sample_indices)` enqueues chunk i for sample
  sample_indices[i] unless that sample has ended; `end(sample_indices=None)`
  enqueues `stop_signal` once per sample and raises its `finished_flags` entry
  (generate() stops at the next step once any flag is up, :443-447).
  `iter(streamer)` yields `{sample: chunk}` dicts until every sample ended;
  `get_stream(i)` iterates one sample.
* `AsyncAudioStreamer`: the same on asyncio queues, fed thread-safely from the
  generating thread through the running loop.

Difference in mechanism only: generate() hands `put` one device block for all
diffusing samples of the step; it is copied to the host ONCE (one D2H per step
instead of one blocking `.cpu()` per sample) and split into per-sample views.
"""
from __future__ import annotations

import asyncio
import queue
import time
from typing import Optional

import torch


def _indices(sample_indices):
    if sample_indices is None:
        return None
    if torch.is_tensor(sample_indices):
        return [int(i) for i in sample_indices.reshape(-1).tolist()]
    return [int(i.item()) if torch.is_tensor(i) else int(i) for i in sample_indices]


def _host_rows(audio_chunks):
    """One host copy of the whole block (rows stay views of it)."""
    if torch.is_tensor(audio_chunks):
        return audio_chunks.detach().cpu()
    return [c.detach().cpu() if torch.is_tensor(c) else c for c in audio_chunks]


class AudioStreamer:
    """Sync per-sample audio queues (reference streamer.py:13-86)."""

    def __init__(self, batch_size: int, stop_signal=None, timeout: Optional[float] = None):
        self.batch_size = batch_size
        self.stop_signal = stop_signal
        self.timeout = timeout
        self.audio_queues = [self._new_queue() for _ in range(batch_size)]
        self.finished_flags = [False] * batch_size
        self.sample_indices_map = {}

    def _new_queue(self):
        return queue.Queue()

    def _enqueue(self, idx, item):
        self.audio_queues[idx].put(item, timeout=self.timeout)

    def _live(self, idx):
        return 0 <= idx < self.batch_size and not self.finished_flags[idx]

    def put(self, audio_chunks: torch.Tensor, sample_indices: torch.Tensor):
        """Enqueue audio_chunks[i] (moved to the host) for sample sample_indices[i]."""
        idx = _indices(sample_indices)
        if not any(self._live(i) for i in idx):
            return
        rows = _host_rows(audio_chunks)
        for i, s in enumerate(idx):
            if self._live(s):
                self._enqueue(s, rows[i])

    def end(self, sample_indices: Optional[torch.Tensor] = None):
        """Signal the end of the given samples (all when None), once each."""
        idx = range(self.batch_size) if sample_indices is None else _indices(sample_indices)
        for s in idx:
            if self._live(s):
                self._enqueue(s, self.stop_signal)
                self.finished_flags[s] = True

    def _is_stop(self, value):
        if self.stop_signal is None or torch.is_tensor(value):
            return value is self.stop_signal
        return value == self.stop_signal

    def __iter__(self):
        return AudioBatchIterator(self)

    def get_stream(self, sample_idx: int):
        if sample_idx >= self.batch_size:
            raise ValueError(f"Sample index {sample_idx} exceeds batch size {self.batch_size}")
        return AudioSampleIterator(self, sample_idx)


class AudioSampleIterator:
    """Chunks of one sample until its stop signal (reference :89-103)."""

    def __init__(self, streamer: AudioStreamer, sample_idx: int):
        self.streamer, self.sample_idx = streamer, sample_idx

    def __iter__(self):
        return self

    def __next__(self):
        value = self.streamer.audio_queues[self.sample_idx].get(timeout=self.streamer.timeout)
        if self.streamer._is_stop(value):
            raise StopIteration
        return value


class AudioBatchIterator:
    """`{sample: chunk}` for the samples that have a chunk ready, polling until
    every sample has ended (reference :106-147)."""

    poll_s = 0.01

    def __init__(self, streamer: AudioStreamer):
        self.streamer = streamer
        self.active_samples = set(range(streamer.batch_size))

    def __iter__(self):
        return self

    def __next__(self):
        while self.active_samples:
            ready, done = {}, set()
            for idx in sorted(self.active_samples):
                try:
                    value = self.streamer.audio_queues[idx].get(block=False)
                except queue.Empty:
                    continue
                if self.streamer._is_stop(value):
                    done.add(idx)
                else:
                    ready[idx] = value
            self.active_samples -= done
            if ready:
                return ready
            if self.active_samples:
                time.sleep(self.poll_s)
        raise StopIteration


class AsyncAudioStreamer(AudioStreamer):
    """asyncio flavour (reference :150-203).  Construct it inside a running
    event loop; generate() may run in a worker thread: every queue operation is
    scheduled on that loop with call_soon_threadsafe."""

    def __init__(self, batch_size: int, stop_signal=None, timeout: Optional[float] = None):
        self.loop = asyncio.get_running_loop()
        super().__init__(batch_size, stop_signal, timeout)

    def _new_queue(self):
        return asyncio.Queue()

    def _enqueue(self, idx, item):
        self.loop.call_soon_threadsafe(self.audio_queues[idx].put_nowait, item)

    async def get_stream(self, sample_idx: int):
        if sample_idx >= self.batch_size:
            raise ValueError(f"Sample index {sample_idx} exceeds batch size {self.batch_size}")
        while True:
            value = await self.audio_queues[sample_idx].get()
            if self._is_stop(value):
                break
            yield value

    def __aiter__(self):
        return AsyncAudioBatchIterator(self)


class AsyncAudioBatchIterator:
    """Async `{sample: chunk}` batches: waits for the first ready sample, then
    also takes whatever the other samples have queued (reference :206-264)."""

    def __init__(self, streamer: AsyncAudioStreamer):
        self.streamer = streamer
        self.active_samples = set(range(streamer.batch_size))

    def __aiter__(self):
        return self

    async def __anext__(self):
        st = self.streamer
        while self.active_samples:
            tasks = {idx: asyncio.ensure_future(st.audio_queues[idx].get()) for idx in sorted(self.active_samples)}
            done, pending = await asyncio.wait(tasks.values(), return_when=asyncio.FIRST_COMPLETED,
                                               timeout=st.timeout)
            for t in pending:
                t.cancel()
            if pending:
                await asyncio.gather(*pending, return_exceptions=True)
            ready, ended = {}, set()
            for idx, t in tasks.items():
                if t not in done or t.cancelled():
                    continue
                value = t.result()
                if st._is_stop(value):
                    ended.add(idx)
                else:
                    ready[idx] = value
            self.active_samples -= ended
            if ready:
                return ready
            if not done:                      # timed out with nothing ready
                raise asyncio.TimeoutError
        raise StopAsyncIteration


__all__ = ["AudioStreamer", "AsyncAudioStreamer", "AudioSampleIterator", "AudioBatchIterator",
           "AsyncAudioBatchIterator"]
