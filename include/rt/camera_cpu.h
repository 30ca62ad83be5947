// camera_cpu.h -- the reference's camera slot (src/camera_cpu.h: CPUImpl::Camera).
//
// This drop-in has no CPU renderer: code written against the reference (src/main.cpp,
// tests/tests.cpp) names CPUImpl::Camera and gets the MI355X camera, so it compiles
// unchanged and renders on the GPU.
#pragma once
#include "camera_hip.h"

namespace CPUImpl {
using Camera = HIPImpl::Camera;
}
