// Test model only — the declaration of Modules/Utils/Geometry.h:115 that the adapter replaces.
#pragma once

#include <memory>

#include "Map/Map.h"
#include "Utils/CommonTypes.h"

void calculatePixelsStandDev(std::shared_ptr<Map> Map, PixelsError &pixelsErrors);
