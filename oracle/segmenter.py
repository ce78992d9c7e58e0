"""Oracle (test infrastructure only): CPU restatement of the reference engine's phrase
segmentation and playback ducking, for checking janus_amd.streaming / janus_amd.receiver.

segment(): the body of smart_ear_loop's while-loop (backend/services/engine.py:445-506)
run over a recorded sequence of chunks, with control_state.is_recording /
is_streaming / mode given per chunk and the VAD decision given per chunk (vad.py is a
remote silero model; the tests supply decisions). Returns (chunk index, phrase audio) for
every phrase handed to process_audio_blocking, i.e. after the 9216-sample skip (:504).

duck(): apply_ducking_if_needed (engine.py:94-134) on int16 PCM bytes, as written there.
Parity: pinned by the reference's own tests only for the behaviours they assert
(test_engine.py:16-101 ducking cases); the segmentation loop is parity unpinned against
reference outputs (its tests mock the loop's services) and follows the source lines.
"""
from collections import deque

import numpy as np


def segment(chunks, speech, recording=None, streaming=None, non_vad=None):
    n = len(chunks)
    recording = recording if recording is not None else [False] * n
    streaming = streaming if streaming is not None else [True] * n
    non_vad = non_vad if non_vad is not None else [False] * n
    audio_buffer = []
    pre_roll_buffer = deque(maxlen=10)
    silence_counter = 0
    SILENCE_THRESHOLD_CHUNKS = 15
    previous_hold_state = False
    out = []
    for i, chunk in enumerate(chunks):
        trigger_processing = False
        if recording[i]:
            audio_buffer.append(chunk)
            previous_hold_state = True
            continue
        if previous_hold_state and not recording[i]:
            trigger_processing = True
            previous_hold_state = False
        elif streaming[i]:
            is_speech = speech[i] or non_vad[i]
            if is_speech:
                if len(audio_buffer) == 0:
                    audio_buffer.extend(list(pre_roll_buffer))
                audio_buffer.append(chunk)
                silence_counter = 0
            else:
                silence_counter += 1
                if len(audio_buffer) > 0:
                    audio_buffer.append(chunk)
                else:
                    pre_roll_buffer.append(chunk)
                if silence_counter > SILENCE_THRESHOLD_CHUNKS:
                    trigger_processing = True
        if trigger_processing and len(audio_buffer) > 0:
            combined_audio = np.concatenate(audio_buffer)
            audio_buffer = []
            silence_counter = 0
            if len(combined_audio) < 1536 * 6:
                continue
            out.append((i, combined_audio))
    return out


def duck(audio_bytes: bytes, ducking_enabled=True, is_talking=False, ducking_level=0.25) -> bytes:
    if not ducking_enabled:
        return audio_bytes
    if not is_talking:
        return audio_bytes
    level = float(ducking_level)
    if level <= 0.0:
        level = 0.0
    elif level >= 1.0:
        return audio_bytes
    if not audio_bytes:
        return audio_bytes
    samples = np.frombuffer(audio_bytes, dtype=np.int16)
    if samples.size == 0:
        return audio_bytes
    scaled = np.clip(samples.astype(np.float32) * level, -32768, 32767).astype(np.int16)
    return scaled.tobytes()
