"""janus_amd — MI355X-native (gfx950) hot path of the Janus semantic voice codec.

Drop-in mirrors of the reference's service classes live in ``janus_amd.services``
(Transcriber, ProsodyExtractor, Synthesizer) and ``janus_amd.common.protocol``
(JanusMode, JanusPacket). All compute goes through ``libjanus_hip.so``
(include/janus.h); there is no CPU fallback.
"""
__version__ = "0.1.0"
