// trt_vocoder.h — boundary shim: the reference's src/trt_vocoder.h is replaced by the MI355X component header.
#pragma once
#include "qwen3_tts_hip.h"
