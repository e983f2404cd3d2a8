"""Reference path vibevoice/modular/streamer.py."""
from vibevoice_amd.streamer import AsyncAudioStreamer, AudioStreamer  # noqa: F401

__all__ = ["AudioStreamer", "AsyncAudioStreamer"]
