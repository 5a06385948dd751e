"""spittle_amd -- MI355X-native (gfx950) Whisper and Parakeet-V3 transcription backend for Spittle.

The hot path (log-mel, encoder, cross-attention K/V, greedy decoder loop) is
hand-written HIP in spittle_amd/csrc, exported through the C ABI in
include/spittle_hip.h (libspittle_hip.so).  This package is the Python mirror of
the transcribe-rs WhisperEngine surface the app binds to.
"""
from .engine import (TranscriptionError, TranscriptionResult, TranscriptionSegment, WhisperEngine,
                     WhisperInferenceParams, WhisperModelParams)

from .parakeet import (ParakeetEngine, ParakeetInferenceParams, ParakeetModelParams, ParakeetResult,
                       TimestampGranularity)

__all__ = ["ParakeetEngine", "ParakeetInferenceParams", "ParakeetModelParams", "ParakeetResult",
           "TimestampGranularity", "WhisperEngine", "WhisperInferenceParams", "WhisperModelParams", "TranscriptionResult",
           "TranscriptionSegment", "TranscriptionError"]
