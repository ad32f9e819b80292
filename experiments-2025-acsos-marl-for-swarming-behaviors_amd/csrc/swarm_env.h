// swarm_env.h — one agent's VMAS World.step + scenario reward, and argmax.
//
// VMAS 1.4.0 World.step restated; scenario rewards:
// go_to_position_scenario.py:108-122, obstacle_avoidance_scenario.py:135-152.
#pragma once
#include "swarm_common.h"

namespace swarm {

struct StepOut {
  float px, py, vx, vy;   // new state
  float dgoal;            // distance to goal after the step
  float dobs;             // World.get_distance(agent, obstacle) (OA)
};

// Drag + Euler and the scenario distances of one agent after its force sum (VMAS
// World._integrate_state, dt 0.1, drag 0.25, mass 1).
__device__ inline StepOut integrate(float px, float py, float vx, float vy, float fx, float fy) {
  StepOut o;
  o.vx = vx * kDragKeep;
  o.vy = vy * kDragKeep;
  o.vx = o.vx + (fx / 1.0f) * kDt;
  o.vy = o.vy + (fy / 1.0f) * kDt;
  o.px = px + o.vx * kDt;
  o.py = py + o.vy * kDt;
  o.dgoal = norm2(o.px - kGoalX, o.py - kGoalY);
  o.dobs = (norm2(o.px - kObstX, o.py - kObstY) - kRadius) - kRadius;
  return o;
}

// OA per-agent reward (obstacle_avoidance_scenario.py:146-152)
__device__ inline float oa_reward(float dgoal, float dobs) {
  const float obst = dobs <= 1.0f ? -(1.0f - dobs) : 0.0f;
  return -dgoal + 2.5f * obst;
}

// torch.argmax: first index of the maximum (train_gcn_dqn.py:168, simulator.py:64)
__device__ inline int argmax9(const float q[kActions]) {
  int best = 0;
  float bv = q[0];
#pragma unroll
  for (int a = 1; a < kActions; ++a)
    if (q[a] > bv) { bv = q[a]; best = a; }
  return best;
}

}  // namespace swarm
