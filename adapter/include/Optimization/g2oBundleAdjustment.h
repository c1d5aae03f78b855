// Declarations of the reference's optimizer API (Modules/Optimization/g2oBundleAdjustment.h:36-75),
// for building the adapter in this repository.  Every signature, parameter type and default
// argument is the reference's, so Modules/System (SLAM.cc:127,145) and Modules/Mapping call the
// adapter exactly as they call g2oBundleAdjustment.cc today.  In the reference tree this file is
// not needed: the reference's own header declares the same functions, and adapter/src/*.cc replaces
// g2oBundleAdjustment.cc as their definition.  Only the Open3D include is absent: getInvUncertainty's
// mesh type is forward-declared (its single call site, g2oBundleAdjustment.cc:887, lies in the
// replaced arapOptimization body, whose result it never used).
#ifndef SLAM_G2OBUNDLEADJUSTMENT_H
#define SLAM_G2OBUNDLEADJUSTMENT_H

#include <cstddef>
#include <memory>
#include <vector>

#include "Map/Map.h"
#include "Mapping/Frame.h"
#include "System/Settings.h"
#include "Visualization/MapVisualizer.h"

namespace open3d::geometry {
class TriangleMesh;
}

// BlockSolver_6_3 bundle adjustment over every KeyFrame and MapPoint (:38-138)
void bundleAdjustment(Map *pMap);

// pose-only optimization of one Frame; outlier MapPoints are removed, the inlier count returned (:140-243)
int poseOnlyOptimization(Frame &currFrame);

// local bundle adjustment around one KeyFrame (:245-444)
void localBundleAdjustment(Map *pMap, ID currKeyFrameId);

// the outer loop: rounds of arapOptimization, optionally with the NLopt weight search (:446-606)
void deformationOptimization(std::shared_ptr<Map> pMap, Settings &settings,
                             std::shared_ptr<MapVisualizer> &mapVisualizer,
                             const std::vector<Eigen::Vector3f> originalPoints = {},
                             const std::vector<Eigen::Vector3f> movedPoints = {});

// the ARAP + reprojection + depth graph of every keyframe pair, solved by LM (:608-1008)
void arapOptimization(Map *pMap, double repBalanceWeight, double globalBalanceWeight, double arapBalanceWeight,
                      double alphaWeight, double betaWeight, float DepthError, int nOptIterations,
                      double *optimizationUpdate = nullptr);

// Open3D's DeformAsRigidAsPossible (:1010-): out of scope, reports and leaves the map unchanged
void arapOpen3DOptimization(Map *pMap);

double getInvUncertainty(std::shared_ptr<open3d::geometry::TriangleMesh> mesh, std::vector<Eigen::Vector3d> v1Positions,
                         std::vector<Eigen::Vector3d> v2Positions, size_t i);

#endif  // SLAM_G2OBUNDLEADJUSTMENT_H
