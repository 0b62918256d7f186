// audio_tokenizer_encoder.h — boundary shim: the reference's src/audio_tokenizer_encoder.h is replaced by the MI355X component header.
#pragma once
#include "qwen3_tts_hip.h"
