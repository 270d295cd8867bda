"""Drop-in for src/contrastor/utils.py (clustering for ProtoNCE / HProtoNCE).

``extract_all_emb`` keeps the reference behaviour (utils.py:11-25: anchor then
positive embedding blocks per batch).  ``run_kmeans`` (utils.py:50-110) runs
Lloyd k-means on the irc HIP kernels (irc_amd.cluster.kmeans) where the
reference uses faiss, then the reference's concentration estimate;
``run_hierarchical_clustering`` (utils.py:112-160) keeps the reference's host
Ward linkage (scipy's implementation of the method fastcluster provides) and
cluster statistics.
"""
import numpy as np
import torch

from irc_amd import cluster


def extract_all_emb(loader, model, device):
    emb_lst = []
    print("[Runner] - Extracting sentence embedding vectors")
    with torch.no_grad():
        for _, anchor_sample, positive_sample in loader:
            a, p = model.bert_extract(anchor_sample, positive_sample, device)
            emb_lst.append(model.seq2vec(a).cpu().numpy())
            emb_lst.append(model.seq2vec(p).cpu().numpy())
    return np.vstack(emb_lst)


def run_kmeans(proto_nce_config, loader, model, device):
    x = extract_all_emb(loader, model, device)
    return kmeans_results(proto_nce_config, x, device)


def kmeans_results(proto_nce_config, x, device):
    """utils.py:55-110 from the embedding matrix x [n, D]."""
    print("[Runner] - Performing kmeans clustering")
    cfg = proto_nce_config["cluster"]
    results = {"emb2cluster": [], "centroids": [], "density": []}
    xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device)
    for seed, num_cluster in enumerate(cfg["num_cluster"]):
        k = int(num_cluster)
        centroids, assign, dist = cluster.kmeans(
            xt, k, niter=int(cfg["niter"]), nredo=int(cfg["nredo"]), seed=seed,
            max_points_per_centroid=int(cfg["max_points_per_centroid"]))
        density = cluster.concentration(assign.cpu().numpy(), dist.cpu().numpy(), k,
                                        proto_nce_config["temperature"])
        centroids = torch.nn.functional.normalize(centroids, p=2, dim=1)
        results["centroids"].append(centroids)
        results["density"].append(torch.tensor(density, dtype=torch.float32, device=device))
        results["emb2cluster"].append(assign)
    return results


def run_hierarchical_clustering(proto_nce_config, loader, model, device):
    import scipy.cluster.hierarchy as sch

    x = extract_all_emb(loader, model, device)
    print("[Runner] - Performing hierarchical clustering")
    results = {"emb2cluster": [], "centroids": [], "density": []}
    dis = sch.linkage(x, metric="euclidean", method="ward")
    for num_cluster in proto_nce_config["cluster"]["num_cluster"]:
        emb2cluster = sch.fcluster(dis, num_cluster, criterion="maxclust") - 1
        centroids, dists = [], np.zeros(len(x))
        for c in range(num_cluster):
            members = np.nonzero(emb2cluster == c)[0]
            cen = x[members].mean(axis=0) if len(members) else np.zeros(x.shape[1])
            centroids.append(cen)
            dists[members] = np.sum((x[members] - cen) ** 2, axis=1)
        density = cluster.concentration(emb2cluster, dists, num_cluster,
                                        proto_nce_config["temperature"])
        centroids = torch.from_numpy(np.array(centroids)).float().to(device)
        results["centroids"].append(torch.nn.functional.normalize(centroids, p=2, dim=1))
        results["density"].append(torch.tensor(density, dtype=torch.float32, device=device))
        results["emb2cluster"].append(torch.as_tensor(emb2cluster, dtype=torch.long,
                                                      device=device))
    return results
