// dccrg.hpp -- the drop-in name: code written against the reference's
// dccrg.hpp (#include "dccrg.hpp") builds against the MI355X implementation.
#ifndef DCCRG_HPP
#define DCCRG_HPP
#include "dccrg_amd.hpp"
#endif
