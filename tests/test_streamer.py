"""AudioStreamer / AsyncAudioStreamer queue protocol (CPU; reference
vibevoice/modular/streamer.py:13-264): put skips ended samples, end signals
each sample once and raises finished_flags, the batch iterator yields
{sample: chunk} until all ended, get_stream iterates one sample, and the async
flavour is fed from another thread as generate() does under gradio."""
import asyncio
import threading

import pytest
import torch

from vibevoice_amd.streamer import AsyncAudioStreamer, AudioStreamer


def _chunks(n, hop=8, base=0.0):
    return torch.arange(n * hop, dtype=torch.float32).reshape(n, 1, hop) + base


def test_put_end_and_sample_stream():
    st = AudioStreamer(3)
    st.put(_chunks(2), torch.tensor([0, 2]))
    st.put(_chunks(1, base=100), torch.tensor([2]))
    st.end(torch.tensor([2]))
    st.put(_chunks(1, base=200), torch.tensor([2]))          # ended: dropped
    assert st.finished_flags == [False, False, True]
    got = list(st.get_stream(2))
    assert len(got) == 2 and torch.equal(got[0], _chunks(2)[1]) and torch.equal(got[1], _chunks(1, base=100)[0])
    assert got[0].device.type == "cpu" and got[0].shape == (1, 8)
    st.end()
    st.end()                                                   # idempotent
    assert st.finished_flags == [True] * 3
    assert [c.shape for c in st.get_stream(0)] == [(1, 8)]
    assert list(st.get_stream(1)) == []
    with pytest.raises(ValueError):
        st.get_stream(3)


def test_batch_iterator_until_all_ended():
    st = AudioStreamer(2)
    st.put(_chunks(2), [0, 1])
    st.put(_chunks(1, base=5), torch.tensor([1]))
    st.end([0])
    st.end(torch.tensor([1]))
    batches = list(st)
    assert set(batches[0]) == {0, 1}
    assert list(batches[1]) == [1] and torch.equal(batches[1][1], _chunks(1, base=5)[0])
    assert len(batches) == 2


def test_custom_stop_signal_and_threaded_producer():
    st = AudioStreamer(1, stop_signal="STOP", timeout=5.0)

    def produce():
        for k in range(4):
            st.put(_chunks(1, base=k), torch.tensor([0]))
        st.end()
    t = threading.Thread(target=produce)
    t.start()
    got = list(st.get_stream(0))
    t.join()
    assert [float(c[0, 0]) for c in got] == [0.0, 1.0, 2.0, 3.0]


def test_async_streamer_fed_from_worker_thread():
    async def main():
        st = AsyncAudioStreamer(2)

        def produce():
            for k in range(3):
                st.put(_chunks(2, base=10 * k), torch.tensor([0, 1]))
            st.end(torch.tensor([0]))
            st.put(_chunks(1, base=99), torch.tensor([1]))
            st.end()
        t = threading.Thread(target=produce)
        t.start()
        seen = {0: [], 1: []}
        async for batch in st:
            for k, v in batch.items():
                seen[k].append(float(v[0, 0]))
        t.join()
        assert st.finished_flags == [True, True]
        return seen
    seen = asyncio.run(main())
    assert seen[0] == [0.0, 10.0, 20.0]
    assert seen[1] == [8.0, 18.0, 28.0, 99.0]


def test_async_get_stream():
    async def main():
        st = AsyncAudioStreamer(1)
        st.put(_chunks(1), torch.tensor([0]))
        st.end()
        await asyncio.sleep(0)
        return [c async for c in st.get_stream(0)]
    got = asyncio.run(main())
    assert len(got) == 1 and got[0].shape == (1, 8)
