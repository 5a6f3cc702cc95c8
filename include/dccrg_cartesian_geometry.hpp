// dccrg_cartesian_geometry.hpp -- drop-in name: dccrg::Cartesian_Geometry is
// defined in dccrg_amd.hpp.
#ifndef DCCRG_CARTESIAN_GEOMETRY_HPP
#define DCCRG_CARTESIAN_GEOMETRY_HPP
#include "dccrg_amd.hpp"
#endif
