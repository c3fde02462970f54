// Synthetic benchmark frames.
#pragma once

#include <stdint.h>

namespace gz {

// rgb: 3*w*h bytes, interleaved.
void SyntheticFrame(uint64_t seed, int w, int h, uint8_t* rgb);

}  // namespace gz
