// text_tokenizer.h — boundary shim: the reference's src/text_tokenizer.h is replaced by the MI355X component header.
#pragma once
#include "qwen3_tts_hip.h"
