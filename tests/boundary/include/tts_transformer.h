// tts_transformer.h — boundary shim: the reference's src/tts_transformer.h is replaced by the MI355X component header.
#pragma once
#include "qwen3_tts_hip.h"
