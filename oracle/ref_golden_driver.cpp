// ref_golden_driver.cpp -- drives the reference's own compilable sources
// (src/gripper.cpp, src/slidingwindow.h, compiled from /root/reference by
// oracle/Makefile into oracle/_ref/) to produce golden vectors for the oracle.
// TEST INFRASTRUCTURE ONLY.  Output: whitespace-separated numbers on stdout.
//
// usage: ref_golden gripper < cmds.txt   (lines: op a b c, ops as or_grip_step_sequence)
//        ref_golden window               (SlidingWindow read_element / read sequences)
#include <cstdio>
#include <cstring>
#include <vector>
#include <stdexcept>
#include "gripper.h"
#include "slidingwindow.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (std::strcmp(argv[1], "gripper") == 0) {
    luke::Gripper end, next;
    int op; double a, b, c;
    while (std::scanf("%d %lf %lf %lf", &op, &a, &b, &c) == 4) {
      int ret = 0;
      if (op == 0) ret = end.set_xyz_m_rad(end.x + a, end.th + b, end.z + c);   // move_gripper_target_m_rad
      else if (op == 1) ret = end.set_xyz_m(end.x + a, end.y + b, end.z + c);   // move_gripper_target_m
      else if (op == 2) ret = next.step_to(end, (int)a);                       // update_stepper step_to
      else if (op == 3) { end.reset(); next.reset(); ret = 1; }
      std::printf("%d %.17g %.17g %.17g %.17g %d %d %d %.17g %.17g %.17g %.17g %d %d %d\n", ret,
                  end.x, end.y, end.z, end.th, end.step.x, end.step.y, end.step.z,
                  next.x, next.y, next.z, next.th, next.step.x, next.step.y, next.step.z);
    }
    return 0;
  }
  if (std::strcmp(argv[1], "window") == 0) {
    // SensorData windows are SlidingWindow<float>(1000) (mjclass.h:1204)
    luke::SlidingWindow<float> w(1000);
    for (int k = 1; k <= 20; k++) {
      w.add((float)k * 0.5f);
      std::printf("%d", k);
      for (int n = 0; n < 10; n++) std::printf(" %.9g", (double)w.read_element(n));
      std::vector<float> r = w.read(7);
      for (float x : r) std::printf(" %.9g", (double)x);
      std::printf("\n");
    }
    return 0;
  }
  return 2;
}
