// Stand-in restating RegistrationParams (aicp_core/include/aicp_registration/common.hpp:7-23).
#pragma once
#include <string>

struct RegistrationParams {
  std::string type = "";
  float sensorRange = -1;
  float sensorAngularView = -1;
  std::string loadPosesFrom = "";
  std::string initialTransform = "";
  struct PointmatcherRegistrationParams {
    std::string configFileName = "";
    std::string initialTransform = "";
    bool printOutputStatistics = false;
  } pointmatcher;
};
