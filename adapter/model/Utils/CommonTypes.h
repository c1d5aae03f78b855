// Test model only — the two structs of Modules/Utils/CommonTypes.h the API passes.
#pragma once

struct PixelsError {
    double avgc1;    // Average error camera 1
    double avgc2;    // Average error camera 2
    double avg;      // Average error across both cameras
    double desvc1;   // Standard deviation camera 1
    double desvc2;   // Standard deviation camera 2
    double desv;     // Standard deviation across both camera
};

struct PoseData {
    double tx = 0.0, ty = 0.0, tz = 0.0;
    double qx = 0.0, qy = 0.0, qz = 0.0, qw = 1.0;
    bool isValid = false;
};
