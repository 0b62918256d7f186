// audio_tokenizer_decoder.h — boundary shim: the reference's src/audio_tokenizer_decoder.h is replaced by the MI355X component header.
#pragma once
#include "qwen3_tts_hip.h"
