// Test model only — the declarations of Modules/Utils/Measurements.h:17-30 that
// deformationOptimization calls between rounds.  They stay the reference's own (Measurements.cc);
// the model's definitions (model/model.cc) record the call in the experiment file.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "Map/Map.h"

void measureSimAbsoluteMapErrors(const std::shared_ptr<Map> pMap, const std::vector<Eigen::Vector3f> originalPoints,
                                 const std::vector<Eigen::Vector3f> movedPoints, const std::string filePath);
void measureRealAbsoluteMapErrors(const std::shared_ptr<Map> pMap, const std::string filePath);
void measureRelativeMapErrors(std::shared_ptr<Map> pMap, std::string filePath);
