// Compiled model (host side) and the MJCF subset compiler that produces it.
//
// Replaces MuJoCo 2.0's mj_loadXML (called at /root/reference/cmd/basic.cpp:123,
// tst/test_derivatives.cpp:34) for the element/attribute subset used by
// res/{inverted_pendulum,hopper,humanoid}.xml.
// Field names and meaning follow mjModel; the list lives in
// include/ilqg_model_fields.h so the model record has one definition.
#pragma once

#include <string>
#include <vector>

#include "ilqg_model_fields.h"

namespace ilqg {

struct HostModel {
#define ILQG_DECL_I(nm) int nm = 0;
#define ILQG_DECL_F(nm) double nm = 0;
#define ILQG_DECL_FA(nm, cnt) std::vector<double> nm;
#define ILQG_DECL_IA(nm, cnt) std::vector<int> nm;
  ILQG_MODEL_I32_SCALARS(ILQG_DECL_I)
  ILQG_MODEL_F64_SCALARS(ILQG_DECL_F)
  ILQG_MODEL_F64_ARRAYS(ILQG_DECL_FA)
  ILQG_MODEL_I32_ARRAYS(ILQG_DECL_IA)
#undef ILQG_DECL_I
#undef ILQG_DECL_F
#undef ILQG_DECL_FA
#undef ILQG_DECL_IA

  std::string model_name;
  std::vector<std::string> body_names, jnt_names, geom_names, actuator_names;
  int nbuffer_bytes = 0;  // mjData arena size MuJoCo 2.0 would allocate (info only)

  // upper bounds used to size per-evaluation device workspaces
  int maxcon = 0;  // contacts the collision pairs can produce (<= nconmax)
  int maxefc = 0;  // constraint rows (<= njmax)
};

// Parse + compile an MJCF file.  Returns false and fills `err` on failure.
bool compile_mjcf_file(const std::string& path, HostModel& m, std::string& err);
bool compile_mjcf_string(const std::string& xml, HostModel& m, std::string& err);

// mj_setConst at qpos0: body/dof invweight0, stat.meaninertia, subtree masses.
void set_const(HostModel& m);

// Serialize to the model record format of include/ilqg_model_blob.h.
std::vector<unsigned char> write_blob(const HostModel& m);

}  // namespace ilqg
