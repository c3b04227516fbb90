// Stand-in for <octomap/octomap.h>: the interface only passes ColorOcTree pointers.
#pragma once
namespace octomap {
class ColorOcTree;
}
